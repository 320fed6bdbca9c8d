// Shared-memory control-plane mailbox for the single-node parameter server.
//
// RCCL has no any-source receive, so in async mode the server must learn WHICH worker is
// ready (and at which local step) before it posts the matching ncclRecv. The reference does
// this implicitly through gRPC unary calls into a 20-thread pool (reference:
// src/parameter_server/server.py:370-393, ps_pb2_grpc.py:28-121). Here every rank of the node
// maps one POSIX shared-memory segment holding a bounded lock-free MPMC ring (Vyukov
// sequence-number queue) of fixed 32-byte control messages, plus one reply slot per worker.
// Latency is a few microseconds (vs ~100 us for a TCPStore round trip).
#include <errno.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <cstdint>
#include <cstring>

namespace {

constexpr uint64_t kMagic = 0x5053584d424f5831ull;  // "PSXMBOX1"

struct Msg {
  int32_t type, src, a, b;
  int64_t c, d;
};
static_assert(sizeof(Msg) == 32, "msg size");

struct Slot {
  std::atomic<uint64_t> seq;
  Msg msg;
  char pad[64 - 8 - sizeof(Msg)];
};

struct Reply {
  std::atomic<uint64_t> seq;  // bumped by the server when a reply is posted
  Msg msg;
  char pad[64 - 8 - sizeof(Msg)];
};

struct Header {
  uint64_t magic;
  uint32_t capacity, nreply;
  alignas(64) std::atomic<uint64_t> head;
  alignas(64) std::atomic<uint64_t> tail;
  alignas(64) std::atomic<uint32_t> ready;
};

struct Box {
  Header* h;
  Slot* slots;
  Reply* replies;
  size_t bytes;
  int owner;
  char name[128];
};

size_t seg_bytes(uint32_t cap, uint32_t nreply) {
  return sizeof(Header) + (size_t)cap * sizeof(Slot) + (size_t)nreply * sizeof(Reply);
}

void nap(int spins) {
  if (spins < 64) return;
  timespec ts{0, spins < 1024 ? 2000 : 20000};
  nanosleep(&ts, nullptr);
}

double now_s() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}

}  // namespace

extern "C" {

// Create (owner=1) or attach (owner=0) a mailbox. capacity must be a power of two.
void* psx_mbox_open(const char* name, int capacity, int nreply, int owner, double timeout_s) {
  if (capacity <= 0 || (capacity & (capacity - 1))) return nullptr;
  const size_t bytes = seg_bytes((uint32_t)capacity, (uint32_t)nreply);
  int fd = -1;
  if (owner) {
    shm_unlink(name);
    fd = shm_open(name, O_CREAT | O_RDWR | O_EXCL, 0600);
    if (fd < 0) return nullptr;
    if (ftruncate(fd, (off_t)bytes) != 0) {
      close(fd);
      shm_unlink(name);
      return nullptr;
    }
  } else {
    const double t0 = now_s();
    for (int spins = 0;; ++spins) {
      fd = shm_open(name, O_RDWR, 0600);
      if (fd >= 0) {
        struct stat st;
        if (fstat(fd, &st) == 0 && (size_t)st.st_size >= bytes) break;
        close(fd);
        fd = -1;
      }
      if (now_s() - t0 > timeout_s) return nullptr;
      nap(spins + 64);
    }
  }
  void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) return nullptr;
  Box* b = new Box();
  b->h = reinterpret_cast<Header*>(p);
  b->slots = reinterpret_cast<Slot*>((char*)p + sizeof(Header));
  b->replies = reinterpret_cast<Reply*>((char*)p + sizeof(Header) + (size_t)capacity * sizeof(Slot));
  b->bytes = bytes;
  b->owner = owner;
  strncpy(b->name, name, sizeof(b->name) - 1);
  if (owner) {
    b->h->capacity = (uint32_t)capacity;
    b->h->nreply = (uint32_t)nreply;
    b->h->head.store(0);
    b->h->tail.store(0);
    for (int i = 0; i < capacity; ++i) b->slots[i].seq.store((uint64_t)i);
    for (int i = 0; i < nreply; ++i) b->replies[i].seq.store(0);
    std::atomic_thread_fence(std::memory_order_release);
    b->h->magic = kMagic;
    b->h->ready.store(1, std::memory_order_release);
  } else {
    const double t0 = now_s();
    for (int spins = 0; b->h->ready.load(std::memory_order_acquire) != 1 || b->h->magic != kMagic; ++spins) {
      if (now_s() - t0 > timeout_s) {
        munmap(p, bytes);
        delete b;
        return nullptr;
      }
      nap(spins + 64);
    }
  }
  return b;
}

void psx_mbox_close(void* hb) {
  Box* b = reinterpret_cast<Box*>(hb);
  if (!b) return;
  munmap(b->h, b->bytes);
  if (b->owner) shm_unlink(b->name);
  delete b;
}

// Enqueue; returns 0 on success, -1 on timeout (queue full).
int psx_mbox_send(void* hb, int type, int src, int a, int b_, long long c, long long d, double timeout_s) {
  Box* b = reinterpret_cast<Box*>(hb);
  const uint64_t mask = b->h->capacity - 1;
  const double t0 = now_s();
  uint64_t pos = b->h->tail.load(std::memory_order_relaxed);
  for (int spins = 0;; ++spins) {
    Slot& s = b->slots[pos & mask];
    const uint64_t seq = s.seq.load(std::memory_order_acquire);
    const int64_t dif = (int64_t)seq - (int64_t)pos;
    if (dif == 0) {
      if (b->h->tail.compare_exchange_weak(pos, pos + 1, std::memory_order_relaxed)) {
        s.msg = Msg{type, src, a, b_, c, d};
        s.seq.store(pos + 1, std::memory_order_release);
        return 0;
      }
    } else if (dif < 0) {
      if (now_s() - t0 > timeout_s) return -1;
      nap(spins);
      pos = b->h->tail.load(std::memory_order_relaxed);
    } else {
      pos = b->h->tail.load(std::memory_order_relaxed);
    }
  }
}

// Dequeue into out[6] (type, src, a, b, c, d as int64); returns 1 if a message was read,
// 0 on timeout. timeout_s = 0 polls once.
int psx_mbox_recv(void* hb, long long* out, double timeout_s) {
  Box* b = reinterpret_cast<Box*>(hb);
  const uint64_t mask = b->h->capacity - 1;
  const double t0 = now_s();
  uint64_t pos = b->h->head.load(std::memory_order_relaxed);
  for (int spins = 0;; ++spins) {
    Slot& s = b->slots[pos & mask];
    const uint64_t seq = s.seq.load(std::memory_order_acquire);
    const int64_t dif = (int64_t)seq - (int64_t)(pos + 1);
    if (dif == 0) {
      if (b->h->head.compare_exchange_weak(pos, pos + 1, std::memory_order_relaxed)) {
        const Msg m = s.msg;
        s.seq.store(pos + mask + 1, std::memory_order_release);
        out[0] = m.type; out[1] = m.src; out[2] = m.a; out[3] = m.b; out[4] = m.c; out[5] = m.d;
        return 1;
      }
    } else if (dif < 0) {
      if (timeout_s <= 0 || now_s() - t0 > timeout_s) return 0;
      nap(spins);
      pos = b->h->head.load(std::memory_order_relaxed);
    } else {
      pos = b->h->head.load(std::memory_order_relaxed);
    }
  }
}

// Server -> worker reply slot (single producer / single consumer per slot).
int psx_mbox_reply(void* hb, int slot, int type, int a, int b_, long long c, long long d) {
  Box* b = reinterpret_cast<Box*>(hb);
  if (slot < 0 || (uint32_t)slot >= b->h->nreply) return -1;
  Reply& r = b->replies[slot];
  r.msg = Msg{type, 0, a, b_, c, d};
  r.seq.fetch_add(1, std::memory_order_release);
  return 0;
}

// Wait until the reply slot's sequence exceeds `last_seq`; returns the new sequence (0 on timeout).
long long psx_mbox_wait_reply(void* hb, int slot, long long last_seq, long long* out, double timeout_s) {
  Box* b = reinterpret_cast<Box*>(hb);
  if (slot < 0 || (uint32_t)slot >= b->h->nreply) return 0;
  Reply& r = b->replies[slot];
  const double t0 = now_s();
  for (int spins = 0;; ++spins) {
    const uint64_t seq = r.seq.load(std::memory_order_acquire);
    if ((long long)seq > last_seq) {
      const Msg m = r.msg;
      out[0] = m.type; out[1] = m.src; out[2] = m.a; out[3] = m.b; out[4] = m.c; out[5] = m.d;
      return (long long)seq;
    }
    if (now_s() - t0 > timeout_s) return 0;
    nap(spins);
  }
}

}  // extern "C"
