// C ABI of the native RCCL data plane (csrc/comm/rccl_comm.cpp), shared with the native server
// event loop (csrc/server/event_loop.cpp). Calls on one communicator are serialized by an internal
// mutex: RCCL communicators are not safe for concurrent enqueue from several threads.
#pragma once
#include <hip/hip_runtime.h>

extern "C" {
int psx_comm_send(void* h, const void* buf, long count, int dtype, int peer, hipStream_t st);
int psx_comm_recv(void* h, void* buf, long count, int dtype, int peer, hipStream_t st);
int psx_comm_reduce_sum(void* h, const void* send, void* recv, long count, int dtype, int root, hipStream_t st);
int psx_comm_broadcast(void* h, void* buf, long count, int dtype, int root, hipStream_t st);
int psx_comm_reduce_scatter_sum(void* h, const void* send, void* recv, long count, int dtype, hipStream_t st);
int psx_comm_all_gather(void* h, const void* send, void* recv, long count, int dtype, hipStream_t st);
int psx_comm_abort(void* h);
int psx_comm_group_start();
int psx_comm_group_end();
}

// psx dtype codes (parallel/rccl.py DTYPES)
enum PsxDtype { PSX_U8 = 0, PSX_F16 = 1, PSX_F32 = 2, PSX_BF16 = 3, PSX_I32 = 4 };
