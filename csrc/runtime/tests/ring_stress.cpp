// SPSC shm ring stress test ("the ring buffer gets a TSan-built C++ unit test").
// One producer thread pushes N variable-length records (sizes 1 B .. 40 KB, so records wrap
// around the ring and exercise the WRAP marker) through a small ring; the consumer thread,
// using its own handle opened by name, checks sequence numbers and every payload byte.
// Built and run with -fsanitize=thread by tests/test_runtime_native.py.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include <unistd.h>

extern "C" {
void* ring_create(const char* name, uint64_t capacity);
void* ring_open(const char* name);
int ring_push(void* hp, const void* buf, uint32_t len, int64_t timeout_ms);
int64_t ring_pop(void* hp, void* buf, uint64_t cap_buf, int64_t timeout_ms, uint64_t* need_out);
void ring_close_writer(void* hp);
void ring_release(void* hp, int unlink);
}

static uint32_t rec_len(uint32_t i) { return 1 + (i * 2654435761u) % 40000u; }

int main(int argc, char** argv) {
  const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : 20000;
  const std::string name = "/tsamd_stress_" + std::to_string((long)getpid());
  void* w = ring_create(name.c_str(), 1 << 17);  // 128 KB: constant wrap-around
  void* r = ring_open(name.c_str());
  if (!w || !r) { fprintf(stderr, "create/open failed\n"); return 2; }
  int bad = 0;
  std::thread prod([&] {
    std::vector<uint8_t> buf(64 * 1024);
    for (uint32_t i = 0; i < n; ++i) {
      const uint32_t L = rec_len(i);
      for (uint32_t k = 0; k < L; ++k) buf[k] = (uint8_t)(i * 31 + k);
      if (L >= 4) memcpy(buf.data(), &i, 4);
      if (ring_push(w, buf.data(), L, -1) != 0) { bad = 1; return; }
    }
    ring_close_writer(w);
  });
  std::thread cons([&] {
    std::vector<uint8_t> buf(64 * 1024);
    uint64_t need = 0;
    for (uint32_t i = 0;; ++i) {
      const int64_t got = ring_pop(r, buf.data(), buf.size(), -1, &need);
      if (got == -2) {  // closed and drained
        if (i != n) { fprintf(stderr, "early end at %u\n", i); bad = 1; }
        return;
      }
      if (got < 0) { fprintf(stderr, "pop error %lld\n", (long long)got); bad = 1; return; }
      const uint32_t L = rec_len(i);
      if ((uint32_t)got != L) { fprintf(stderr, "len mismatch at %u\n", i); bad = 1; return; }
      uint8_t expect[4];
      memcpy(expect, &i, 4);
      for (uint32_t k = 0; k < L; ++k) {
        const uint8_t e = k < 4 && L >= 4 ? expect[k] : (uint8_t)(i * 31 + k);
        if (buf[k] != e) { fprintf(stderr, "byte mismatch rec %u off %u\n", i, k); bad = 1; return; }
      }
    }
  });
  prod.join();
  cons.join();
  ring_release(r, 0);
  ring_release(w, 1);
  if (!bad) printf("OK %u records\n", n);
  return bad;
}
