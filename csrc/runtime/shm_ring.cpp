// Single-producer / single-consumer record ring in POSIX shared memory.
//
// Replaces Flink-AI-Extended's JVM<->Python mmap queue: the ingestion process (streaming
// source / driver) pushes length-prefixed records (serialized tf.Example rows), each GPU
// worker process pops them; results flow back through a second ring.  The consumer side
// is drained by a dedicated thread in the Python wrapper so results are emitted as soon
// as they are produced (the Issue-6 "results lag one record" fix).
//
// Layout: [Header (256 B, cache-line separated counters)][data: capacity bytes].
// head = bytes ever written, tail = bytes ever read (monotonic uint64, wrap by modulo).
// A record = u32 length + payload, padded to 8 B; a record never straddles the end: if
// it does not fit before the end, a WRAP marker (len = 0xFFFFFFFF) fills the rest.
// Blocking ops poll with exponential backoff (1 us .. 1 ms) and honour a timeout; the
// writer's close() makes a drained reader return -2 (end of stream).
#include <atomic>
#include <cerrno>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <fcntl.h>
#include <string>
#include <sys/mman.h>
#include <sys/stat.h>
#include <thread>
#include <unistd.h>
#include <vector>

namespace {

const uint64_t kMagic = 0x5453414d4452494eull;  // "TSAMDRIN"
const uint32_t kWrap = 0xFFFFFFFFu;

struct alignas(64) Header {
  uint64_t magic;
  uint64_t capacity;
  alignas(64) std::atomic<uint64_t> head;
  alignas(64) std::atomic<uint64_t> tail;
  alignas(64) std::atomic<uint32_t> closed;
  std::atomic<uint64_t> records_in;
  std::atomic<uint64_t> records_out;
};
static_assert(sizeof(Header) <= 256, "header too large");
static_assert(std::atomic<uint64_t>::is_always_lock_free, "need lock-free 64-bit atomics in shared memory");

struct Ring {
  std::string name;
  int fd = -1;
  size_t map_len = 0;
  Header* h = nullptr;
  uint8_t* data = nullptr;
  bool owner = false;
};

inline uint64_t align8(uint64_t x) { return (x + 7) & ~uint64_t(7); }

template <typename Pred>
bool wait_until(Pred ok, int64_t timeout_ms) {
  auto t0 = std::chrono::steady_clock::now();
  int64_t sleep_us = 1;
  while (!ok()) {
    if (timeout_ms >= 0) {
      auto el = std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - t0).count();
      if (el >= timeout_ms) return ok();
    }
    std::this_thread::sleep_for(std::chrono::microseconds(sleep_us));
    sleep_us = sleep_us < 1000 ? sleep_us * 2 : 1000;
  }
  return true;
}

}  // namespace

extern "C" {

void* ring_create(const char* name, uint64_t capacity) {
  capacity = align8(capacity < 4096 ? 4096 : capacity);
  shm_unlink(name);
  int fd = shm_open(name, O_CREAT | O_EXCL | O_RDWR, 0600);
  if (fd < 0) return nullptr;
  size_t len = 256 + capacity;
  if (ftruncate(fd, off_t(len)) != 0) { close(fd); shm_unlink(name); return nullptr; }
  void* m = mmap(nullptr, len, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  if (m == MAP_FAILED) { close(fd); shm_unlink(name); return nullptr; }
  auto* r = new Ring;
  r->name = name; r->fd = fd; r->map_len = len; r->owner = true;
  r->h = new (m) Header();
  r->h->capacity = capacity;
  r->h->head.store(0); r->h->tail.store(0); r->h->closed.store(0);
  r->h->records_in.store(0); r->h->records_out.store(0);
  r->data = static_cast<uint8_t*>(m) + 256;
  std::atomic_thread_fence(std::memory_order_release);
  r->h->magic = kMagic;
  return r;
}

void* ring_open(const char* name) {
  int fd = shm_open(name, O_RDWR, 0600);
  if (fd < 0) return nullptr;
  struct stat st;
  if (fstat(fd, &st) != 0 || st.st_size < 256 + 4096) { close(fd); return nullptr; }
  void* m = mmap(nullptr, size_t(st.st_size), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  if (m == MAP_FAILED) { close(fd); return nullptr; }
  auto* r = new Ring;
  r->name = name; r->fd = fd; r->map_len = size_t(st.st_size);
  r->h = static_cast<Header*>(m);
  if (r->h->magic != kMagic) { munmap(m, r->map_len); close(fd); delete r; return nullptr; }
  r->data = static_cast<uint8_t*>(m) + 256;
  return r;
}

// 0 ok, -1 timeout, -2 closed, -3 record larger than the ring.
int ring_push(void* hp, const void* buf, uint32_t len, int64_t timeout_ms) {
  auto* r = static_cast<Ring*>(hp);
  Header* h = r->h;
  const uint64_t cap = h->capacity;
  const uint64_t need = align8(4 + uint64_t(len));
  if (need + 8 > cap || len == kWrap) return -3;
  if (h->closed.load(std::memory_order_acquire)) return -2;
  uint64_t head = h->head.load(std::memory_order_relaxed);
  uint64_t pos = head % cap;
  uint64_t extra = (pos + need > cap) ? cap - pos : 0;  // wrap padding
  bool ok = wait_until([&] { return head + extra + need - h->tail.load(std::memory_order_acquire) <= cap; },
                       timeout_ms);
  if (!ok) return -1;
  if (extra) {
    uint32_t w = kWrap;
    std::memcpy(r->data + pos, &w, 4);
    head += extra;
    pos = 0;
  }
  std::memcpy(r->data + pos, &len, 4);
  if (len) std::memcpy(r->data + pos + 4, buf, len);
  h->records_in.fetch_add(1, std::memory_order_relaxed);
  h->head.store(head + need, std::memory_order_release);
  return 0;
}

// >=0 length, -1 timeout, -2 closed and drained, -3 buffer too small (*need set).
int64_t ring_pop(void* hp, void* buf, uint64_t cap_buf, int64_t timeout_ms, uint64_t* need_out) {
  auto* r = static_cast<Ring*>(hp);
  Header* h = r->h;
  const uint64_t cap = h->capacity;
  uint64_t tail = h->tail.load(std::memory_order_relaxed);
  for (;;) {
    bool ok = wait_until([&] { return h->head.load(std::memory_order_acquire) != tail ||
                                      h->closed.load(std::memory_order_acquire); }, timeout_ms);
    if (h->head.load(std::memory_order_acquire) == tail) {
      if (h->closed.load(std::memory_order_acquire)) return -2;
      if (!ok) return -1;
      continue;
    }
    uint64_t pos = tail % cap;
    uint32_t len;
    std::memcpy(&len, r->data + pos, 4);
    if (len == kWrap) {
      tail += cap - pos;
      h->tail.store(tail, std::memory_order_release);
      continue;
    }
    if (len > cap_buf) {
      if (need_out) *need_out = len;
      return -3;
    }
    if (len) std::memcpy(buf, r->data + pos + 4, len);
    h->records_out.fetch_add(1, std::memory_order_relaxed);
    h->tail.store(tail + align8(4 + uint64_t(len)), std::memory_order_release);
    return int64_t(len);
  }
}

void ring_close_writer(void* hp) { static_cast<Ring*>(hp)->h->closed.store(1, std::memory_order_release); }
int ring_is_closed(void* hp) { return int(static_cast<Ring*>(hp)->h->closed.load()); }
uint64_t ring_pending_bytes(void* hp) {
  auto* h = static_cast<Ring*>(hp)->h;
  return h->head.load() - h->tail.load();
}
uint64_t ring_records_in(void* hp) { return static_cast<Ring*>(hp)->h->records_in.load(); }
uint64_t ring_records_out(void* hp) { return static_cast<Ring*>(hp)->h->records_out.load(); }
uint64_t ring_capacity(void* hp) { return static_cast<Ring*>(hp)->h->capacity; }

void ring_release(void* hp, int unlink) {
  auto* r = static_cast<Ring*>(hp);
  if (!r) return;
  munmap(reinterpret_cast<void*>(r->h), r->map_len);
  close(r->fd);
  if (unlink) shm_unlink(r->name.c_str());
  delete r;
}

}  // extern "C"

// ---------------------------------------------------------------------------------------------
// Ring pipes: native forwarding threads between rings (no Python, no GIL on the record path).
//
//   fanout: one source ring -> n destination rings; record k goes to dst[(k / group) % n], so
//           with group = rows per batch every destination receives whole, consecutive batches
//           (a stream worker's packer processes each build the batches of their own groups, and
//           the trainer reads the packers' outputs round-robin: the serial batch order);
//           end of stream at the source closes every destination.
//   fanin:  n source rings -> one destination ring, each record forwarded the moment it lands
//           (whichever source has one: emit-immediately, Issue-6); the destination is closed
//           once every source is closed and drained (if close_dst).
// Both poll with the rings' own backoff; ring_pipe_stop() makes them exit within ~50 ms.
namespace {

struct Pipe {
  std::thread th;
  std::atomic<int> stop{0};
  std::atomic<int64_t> count{0};
  std::atomic<int> err{0};  // 0 ok, -2 a destination was closed by its consumer, -4 source pop error
};

// blocking push that honours the stop flag; false when stopped or the destination closed
bool pipe_push(Pipe* p, void* dst, const void* buf, uint32_t len) {
  for (;;) {
    int rc = ring_push(dst, buf, len, 50);
    if (rc == 0) return true;
    if (rc == -2 || rc == -3) {
      p->err.store(rc, std::memory_order_relaxed);
      return false;
    }
    if (p->stop.load(std::memory_order_relaxed)) return false;
  }
}

// pop into a growable buffer: >= 0 length, -1 timeout, -2 closed and drained
int64_t pipe_pop(void* src, std::string& buf, int64_t timeout_ms) {
  for (;;) {
    uint64_t need = 0;
    int64_t n = ring_pop(src, &buf[0], buf.size(), timeout_ms, &need);
    if (n != -3) return n;
    buf.resize(size_t(need) * 2);
  }
}

void fanout_main(Pipe* p, void* src, std::vector<void*> dsts, int64_t group) {
  std::string buf(1 << 16, '\0');
  const int64_t n = int64_t(dsts.size());
  int64_t k = 0;
  while (!p->stop.load(std::memory_order_relaxed)) {
    int64_t len = pipe_pop(src, buf, 50);
    if (len == -1) continue;
    if (len < 0) break;  // end of stream
    if (!pipe_push(p, dsts[size_t((k / group) % n)], buf.data(), uint32_t(len))) break;
    ++k;
    p->count.store(k, std::memory_order_relaxed);
  }
  for (void* d : dsts) ring_close_writer(d);
}

void fanin_main(Pipe* p, std::vector<void*> srcs, void* dst, int close_dst) {
  std::string buf(1 << 16, '\0');
  std::vector<char> live(srcs.size(), 1);
  size_t nlive = srcs.size();
  int64_t k = 0, idle_us = 1;
  while (nlive && !p->stop.load(std::memory_order_relaxed)) {
    bool any = false;
    for (size_t i = 0; i < srcs.size(); ++i) {
      if (!live[i]) continue;
      int64_t len = pipe_pop(srcs[i], buf, 0);
      if (len == -1) continue;
      if (len < 0) {  // closed and drained
        live[i] = 0;
        --nlive;
        continue;
      }
      any = true;
      if (!pipe_push(p, dst, buf.data(), uint32_t(len))) { nlive = 0; break; }
      p->count.store(++k, std::memory_order_relaxed);
    }
    if (any) {
      idle_us = 1;
    } else if (nlive) {
      std::this_thread::sleep_for(std::chrono::microseconds(idle_us));
      idle_us = idle_us < 500 ? idle_us * 2 : 500;
    }
  }
  if (close_dst) ring_close_writer(dst);
}

}  // namespace

extern "C" {

void* ring_fanout_start(void* src, void** dsts, int n, int64_t group) {
  if (!src || n < 1 || group < 1) return nullptr;
  auto* p = new Pipe;
  p->th = std::thread(fanout_main, p, src, std::vector<void*>(dsts, dsts + n), group);
  return p;
}

void* ring_fanin_start(void** srcs, int n, void* dst, int close_dst) {
  if (!dst || n < 1) return nullptr;
  auto* p = new Pipe;
  p->th = std::thread(fanin_main, p, std::vector<void*>(srcs, srcs + n), dst, close_dst);
  return p;
}

int64_t ring_pipe_count(void* hp) { return static_cast<Pipe*>(hp)->count.load(); }
void ring_pipe_stop(void* hp) { static_cast<Pipe*>(hp)->stop.store(1); }

// join and free: records forwarded, or the (negative) error
int64_t ring_pipe_join(void* hp) {
  auto* p = static_cast<Pipe*>(hp);
  if (p->th.joinable()) p->th.join();
  const int e = p->err.load();
  const int64_t c = p->count.load();
  delete p;
  return e ? int64_t(e) : c;
}

}  // extern "C"
