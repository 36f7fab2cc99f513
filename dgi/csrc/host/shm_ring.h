// Node-local control plane core: single-producer / single-consumer message rings
// in POSIX shared memory.  Header-only so the pybind11 module (shm_ring.cc) and the
// sanitizer stress driver (shm_ring_stress.cc, built with ASan+UBSan and with TSan by
// ``python -m dgi.build --sanitize``) compile the same code.
//
// Layout (all offsets 8-byte aligned, capacity a power of two):
//   Header | data[capacity]
//   message = u64 length | payload | pad to 8 bytes   (may wrap around the end)
// head / tail are monotonically increasing byte counters on their own cache
// lines; the producer publishes with a release store of head after copying the
// payload, the consumer frees space with a release store of tail after copying
// it out.
#pragma once

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

// Memory order of the cursor publications.  Release is the protocol; the sanitizer self-test
// (tests/test_control_plane.py) rebuilds the TSan driver with relaxed publications and expects
// TSan to report the payload race that opens up.
#ifndef DGI_SHM_PUBLISH_ORDER
#define DGI_SHM_PUBLISH_ORDER std::memory_order_release
#endif

namespace dgi_shm {

constexpr uint64_t kMagic = 0x676e69722d696764ULL;  // "dgi-ring"

struct Header {
  alignas(64) std::atomic<uint64_t> magic;
  uint64_t capacity;
  alignas(64) std::atomic<uint64_t> head;  // bytes published by the producer
  alignas(64) std::atomic<uint64_t> tail;  // bytes released by the consumer
  alignas(64) std::atomic<uint64_t> messages;
};
static_assert(std::atomic<uint64_t>::is_always_lock_free, "shared-memory cursors must be lock-free");
constexpr size_t kHeaderBytes = 256;
static_assert(sizeof(Header) <= kHeaderBytes, "header overflows its reserved bytes");

inline uint64_t round8(uint64_t n) { return (n + 7) & ~uint64_t(7); }

inline void cpu_relax() {
#if defined(__x86_64__)
  __builtin_ia32_pause();
#endif
}

// Escalating wait: spin, then yield, then short sleeps.  Returns false on timeout.
template <class Ready>
bool wait_until(Ready ready, double timeout_s) {
  using clk = std::chrono::steady_clock;
  const auto t0 = clk::now();
  for (int i = 0;; ++i) {
    if (ready()) return true;
    if (i < 256) {
      cpu_relax();
    } else if (i < 1024) {
      std::this_thread::yield();
    } else {
      std::this_thread::sleep_for(std::chrono::microseconds(i < 4096 ? 5 : 50));
      if (timeout_s >= 0 &&
          std::chrono::duration<double>(clk::now() - t0).count() > timeout_s) {
        return ready();
      }
    }
  }
}

class Ring {
 public:
  // producer side: create (fails if the name exists)
  static Ring* create(const std::string& name, uint64_t capacity) {
    if (capacity < 4096 || (capacity & (capacity - 1)) != 0)
      throw std::invalid_argument("ring capacity must be a power of two >= 4096");
    int fd = shm_open(name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
    if (fd < 0) throw std::runtime_error("shm_open(create) " + name + ": " + std::strerror(errno));
    size_t bytes = kHeaderBytes + capacity;
    if (ftruncate(fd, static_cast<off_t>(bytes)) != 0) {
      int e = errno;
      close(fd);
      shm_unlink(name.c_str());
      throw std::runtime_error("ftruncate " + name + ": " + std::strerror(e));
    }
    Ring* r = new Ring(name, fd, bytes, true);
    r->h_->capacity = capacity;
    r->h_->head.store(0, std::memory_order_relaxed);
    r->h_->tail.store(0, std::memory_order_relaxed);
    r->h_->messages.store(0, std::memory_order_relaxed);
    r->h_->magic.store(kMagic, std::memory_order_release);
    return r;
  }

  // consumer side: open if the producer has created and initialised it, else nullptr
  static Ring* try_open(const std::string& name) {
    int fd = shm_open(name.c_str(), O_RDWR, 0600);
    if (fd < 0) return nullptr;
    struct stat st;
    if (fstat(fd, &st) != 0 || static_cast<size_t>(st.st_size) <= kHeaderBytes) {
      close(fd);
      return nullptr;
    }
    Ring* r = new Ring(name, fd, static_cast<size_t>(st.st_size), false);
    if (r->h_->magic.load(std::memory_order_acquire) != kMagic) {
      delete r;
      return nullptr;
    }
    return r;
  }

  ~Ring() {
    if (base_ != nullptr) munmap(base_, bytes_);
    if (fd_ >= 0) close(fd_);
  }

  uint64_t capacity() const { return h_->capacity; }
  uint64_t pending_bytes() const {
    return h_->head.load(std::memory_order_acquire) - h_->tail.load(std::memory_order_acquire);
  }
  uint64_t messages() const { return h_->messages.load(std::memory_order_relaxed); }
  const std::string& name() const { return name_; }

  // false if the ring has no room for the message right now
  bool try_write(const char* p, uint64_t n) {
    const uint64_t cap = h_->capacity;
    const uint64_t need = 8 + round8(n);
    if (need > cap / 2) throw std::length_error("message of " + std::to_string(n) + " bytes exceeds ring " + name_);
    const uint64_t head = h_->head.load(std::memory_order_relaxed);
    const uint64_t tail = h_->tail.load(std::memory_order_acquire);
    if (cap - (head - tail) < need) return false;
    const uint64_t o = head & (cap - 1);
    std::memcpy(data_ + o, &n, 8);  // 8-aligned and cap is a multiple of 8: never straddles
    copy_in(o + 8, p, n);
    h_->messages.fetch_add(1, std::memory_order_relaxed);
    h_->head.store(head + need, DGI_SHM_PUBLISH_ORDER);
    return true;
  }

  bool write(const char* p, uint64_t n, double timeout_s) {
    if (try_write(p, n)) return true;
    return wait_until([&] { return try_write(p, n); }, timeout_s);
  }

  bool has_message() const {
    return h_->head.load(std::memory_order_acquire) != h_->tail.load(std::memory_order_relaxed);
  }

  // caller checked has_message(); copies the payload out and releases it
  std::string read_one() {
    const uint64_t cap = h_->capacity;
    const uint64_t tail = h_->tail.load(std::memory_order_relaxed);
    const uint64_t o = tail & (cap - 1);
    uint64_t n;
    std::memcpy(&n, data_ + o, 8);
    std::string out(n, '\0');
    copy_out(o + 8, &out[0], n);
    h_->tail.store(tail + 8 + round8(n), DGI_SHM_PUBLISH_ORDER);
    return out;
  }

 private:
  Ring(std::string name, int fd, size_t bytes, bool producer) : name_(std::move(name)), fd_(fd), bytes_(bytes) {
    void* m = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    if (m == MAP_FAILED) {
      close(fd);
      fd_ = -1;
      if (producer) shm_unlink(name_.c_str());
      throw std::runtime_error("mmap " + name_ + ": " + std::strerror(errno));
    }
    base_ = static_cast<char*>(m);
    h_ = reinterpret_cast<Header*>(base_);
    data_ = base_ + kHeaderBytes;
  }

  void copy_in(uint64_t off, const char* src, uint64_t n) {
    const uint64_t cap = h_->capacity;
    off &= cap - 1;
    const uint64_t first = std::min<uint64_t>(n, cap - off);
    std::memcpy(data_ + off, src, first);
    if (n > first) std::memcpy(data_, src + first, n - first);
  }

  void copy_out(uint64_t off, char* dst, uint64_t n) const {
    const uint64_t cap = h_->capacity;
    off &= cap - 1;
    const uint64_t first = std::min<uint64_t>(n, cap - off);
    std::memcpy(dst, data_ + off, first);
    if (n > first) std::memcpy(dst + first, data_, n - first);
  }

  std::string name_;
  int fd_ = -1;
  size_t bytes_ = 0;
  char* base_ = nullptr;
  Header* h_ = nullptr;
  char* data_ = nullptr;
};

}  // namespace dgi_shm
