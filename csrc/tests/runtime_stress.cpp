// Concurrency stress test of the native runtime (csrc/runtime), built and run under
// ThreadSanitizer and AddressSanitizer+UBSan by tests/test_sanitizers.py (host code only —
// GPU sanitizers are not used). It exercises the races the reference server has
// (unlocked counters, staleness read outside the lock, the sync
// double-push overwrite) against psx's core and mailbox:
//   1. sync barrier, 8 threads x R rounds: exactly one APPLY per round, every round has all 8
//      members, a second push in the same round is a DUPLICATE (never counted twice);
//   2. async, 8 threads x N pushes: accepted + rejected == pushes, histogram sum == accepted,
//      global step == number of applied updates;
//   3. shared-memory MPMC mailbox, 8 producers x M request/reply round trips against one
//      consumer: no loss, no duplication, per-producer FIFO order.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <unistd.h>

#include <atomic>
#include <thread>
#include <vector>

#include "../runtime/ps_core.h"

extern "C" {
void* psx_mbox_open(const char* name, int capacity, int nreply, int owner, double timeout_s);
void psx_mbox_close(void* hb);
int psx_mbox_send(void* hb, int type, int src, int a, int b, long long c, long long d, double timeout_s);
int psx_mbox_recv(void* hb, long long* out, double timeout_s);
int psx_mbox_reply(void* hb, int slot, int type, int a, int b, long long c, long long d);
long long psx_mbox_wait_reply(void* hb, int slot, long long last_seq, long long* out, double timeout_s);
}

#define CHECK(c)                                                        \
  do {                                                                  \
    if (!(c)) {                                                         \
      fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      exit(1);                                                          \
    }                                                                   \
  } while (0)

static void sync_barrier(int nthr, int rounds) {
  void* c = psx_ps_create(PSX_SYNC, nthr, 0.1f, 5, PSX_BARRIER);
  for (int w = 0; w < nthr; ++w) CHECK(psx_ps_register(c, "w", w, 0.0) == w);
  std::atomic<int> applies{0}, dups{0};
  std::vector<std::thread> th;
  for (int w = 0; w < nthr; ++w)
    th.emplace_back([&, w] {
      for (int r = 0; r < rounds; ++r) {
        while (psx_ps_global_step(c) < r) std::this_thread::yield();  // fetch the round's params
        float wt;
        int n;
        int64_t s;
        const int d = psx_ps_on_push(c, w, r, 0.0, &wt, &n, &s);
        if (d == PSX_APPLY) {
          CHECK(n == nthr);
          int mem[64];
          CHECK(psx_ps_round_members(c, mem, 64) == nthr);
          applies++;
          psx_ps_on_applied(c, 1e-6);
        } else {
          CHECK(d == PSX_WAIT);
          // an eager second push of the same round is never counted again — also when the
          // round completes in between (stale local step) before its apply bumps the step
          if (r % 7 == 3) {
            const int d2 = psx_ps_on_push(c, w, r, 0.0, &wt, &n, &s);
            CHECK(d2 == PSX_DUPLICATE);
            dups++;
          }
        }
      }
    });
  for (auto& t : th) t.join();
  CHECK(applies == rounds);
  CHECK(psx_ps_global_step(c) == rounds);
  printf("sync barrier: %d rounds x %d workers ok (%d duplicate pushes rejected)\n", rounds, nthr, dups.load());
  psx_ps_destroy(c);
}

static void async_stress(int nthr, int pushes) {
  void* c = psx_ps_create(PSX_ASYNC, nthr, 0.1f, 2, PSX_BARRIER);
  for (int w = 0; w < nthr; ++w) psx_ps_register(c, "w", w, 0.0);
  std::atomic<int> acc{0}, rej{0};
  std::vector<std::thread> th;
  for (int w = 0; w < nthr; ++w)
    th.emplace_back([&, w] {
      int64_t ls = 0;
      for (int i = 0; i < pushes; ++i) {
        if (i % (1 + w % 4) == 0) ls = psx_ps_on_fetch(c, w, 0.0);  // some workers fetch rarely -> stale
        float wt;
        int n;
        int64_t s;
        const int d = psx_ps_on_push(c, w, ls, 0.0, &wt, &n, &s);
        if (d == PSX_APPLY) {
          CHECK(s >= 0 && s <= 2 && wt > 0.f && wt <= 1.f);
          acc++;
          psx_ps_on_applied(c, 1e-6);
        } else {
          CHECK(d == PSX_REJECT && s > 2);
          rej++;
        }
      }
    });
  for (auto& t : th) t.join();
  CHECK(acc + rej == nthr * pushes);
  CHECK(rej > 0 && acc > 0);
  CHECK(psx_ps_global_step(c) == acc);
  int64_t hist[64];
  const int nb = psx_ps_staleness_hist(c, hist, 64);
  int64_t tot = 0;
  for (int i = 0; i < nb; ++i) tot += hist[i];
  CHECK(tot == acc);
  char buf[4096];
  CHECK(psx_ps_metrics_json(c, 1.0, buf, sizeof buf) > 0);
  printf("async: %d pushes, %d applied, %d rejected ok\n", nthr * pushes, acc.load(), rej.load());
  psx_ps_destroy(c);
}

static void mailbox_stress(int nthr, int msgs) {
  char name[64];
  snprintf(name, sizeof name, "/psx_stress_%d", (int)getpid());
  void* srv = psx_mbox_open(name, 64, nthr, 1, 5.0);
  CHECK(srv);
  std::vector<std::thread> th;
  for (int w = 0; w < nthr; ++w)
    th.emplace_back([&, w] {
      void* cli = psx_mbox_open(name, 64, nthr, 0, 5.0);
      CHECK(cli);
      long long last = 0, out[6];
      for (int i = 0; i < msgs; ++i) {
        CHECK(psx_mbox_send(cli, 1, w, i, 0, (long long)w * 1000000 + i, 0, 10.0) == 0);
        const long long seq = psx_mbox_wait_reply(cli, w, last, out, 10.0);
        CHECK(seq > last);
        last = seq;
        CHECK(out[2] == i && out[4] == (long long)w * 1000000 + i + 1);  // reply to *this* request
      }
      psx_mbox_close(cli);
    });
  std::vector<int> next(nthr, 0);
  long long out[6];
  for (long total = 0; total < (long)nthr * msgs;) {
    if (!psx_mbox_recv(srv, out, 1.0)) continue;
    const int src = (int)out[1];
    CHECK(src >= 0 && src < nthr);
    CHECK(out[2] == next[src]);  // per-producer FIFO, no loss / duplication
    next[src]++;
    CHECK(psx_mbox_reply(srv, src, 2, (int)out[2], 0, out[4] + 1, 0) == 0);
    ++total;
  }
  for (auto& t : th) t.join();
  psx_mbox_close(srv);
  printf("mailbox: %d producers x %d request/reply round trips ok\n", nthr, msgs);
}

int main(int argc, char** argv) {
  const int scale = argc > 1 ? atoi(argv[1]) : 1;
  sync_barrier(8, 300 * scale);
  async_stress(8, 2000 * scale);
  mailbox_stress(8, 2000 * scale);
  printf("runtime stress: all ok\n");
  return 0;
}
