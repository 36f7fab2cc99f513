// Sanitizer stress driver for the shared-memory control rings (shm_ring.h).
//
// Built twice by ``python -m dgi.build --sanitize``: once with
// -fsanitize=address,undefined and once with -fsanitize=thread, and run by
// tests/test_control_plane.py and the CI ``sanitizers`` job.  It drives the same
// SPSC protocol the Python tests drive, without an interpreter in the way (a
// sanitized extension module would need its runtime preloaded into python):
//
//   threads  producer and consumer threads on ONE mapping (TSan sees every cursor
//            and payload access of both sides), variable sizes, wrap-around,
//            blocking sends on a small ring (back-pressure)
//   fork     producer in a child process, consumer in the parent, each with its own
//            mapping of the ring (the runtime's layout: one process per rank);
//            ASan/UBSan check every copy against the mapping bounds
//   limits   full ring, timeouts, oversize messages, exact wrap at the end
//
// Exit status 0 and one "ok <mode> <messages>" line per mode on success.
#include "shm_ring.h"

#include <cstdio>
#include <cstdlib>
#include <string>
#include <thread>
#include <vector>

#include <sys/wait.h>

namespace {

using dgi_shm::Ring;

// deterministic message i: length from a small LCG, bytes = (i + j) & 0xff, 8-byte id tail
std::string make_msg(uint64_t i, uint64_t max_len) {
  uint64_t x = i * 6364136223846793005ULL + 1442695040888963407ULL;
  const uint64_t n = (x >> 33) % (max_len + 1);
  std::string s(n + 8, '\0');
  for (uint64_t j = 0; j < n; ++j) s[j] = static_cast<char>((i + j) & 0xff);
  std::memcpy(&s[n], &i, 8);
  return s;
}

[[noreturn]] void fail(const char* mode, const std::string& why) {
  std::fprintf(stderr, "FAIL %s: %s\n", mode, why.c_str());
  std::exit(1);
}

void check(const char* mode, uint64_t i, const std::string& got, uint64_t max_len) {
  const std::string want = make_msg(i, max_len);
  if (got != want) fail(mode, "message " + std::to_string(i) + " differs (" + std::to_string(got.size()) +
                                  " vs " + std::to_string(want.size()) + " bytes)");
}

std::string ring_name(const char* tag) {
  return "/dgi.stress." + std::string(tag) + "." + std::to_string(getpid());
}

void consume(const char* mode, Ring* r, uint64_t n, uint64_t max_len) {
  for (uint64_t i = 0; i < n; ++i) {
    if (!dgi_shm::wait_until([&] { return r->has_message(); }, 60.0)) fail(mode, "consumer timed out");
    check(mode, i, r->read_one(), max_len);
  }
  if (r->has_message()) fail(mode, "extra message");
}

void produce(const char* mode, Ring* w, uint64_t n, uint64_t max_len) {
  for (uint64_t i = 0; i < n; ++i) {
    const std::string m = make_msg(i, max_len);
    if (!w->write(m.data(), m.size(), 60.0)) fail(mode, "producer timed out");
  }
}

int run_threads(uint64_t n) {
  const std::string name = ring_name("thr");
  Ring* w = Ring::create(name, 1 << 14);  // small: the producer blocks on a full ring often
  shm_unlink(name.c_str());
  const uint64_t max_len = 3000;
  std::thread prod([&] { produce("threads", w, n, max_len); });
  consume("threads", w, n, max_len);
  prod.join();
  if (w->messages() != n) fail("threads", "message counter");
  delete w;
  std::printf("ok threads %llu\n", static_cast<unsigned long long>(n));
  return 0;
}

int run_fork(uint64_t n) {
  const std::string name = ring_name("fork");
  const uint64_t max_len = 5000;
  pid_t pid = fork();
  if (pid < 0) fail("fork", "fork failed");
  if (pid == 0) {
    Ring* w = Ring::create(name, 1 << 16);
    produce("fork", w, n, max_len);
    // wait until the consumer drained everything before unmapping our end
    dgi_shm::wait_until([&] { return w->pending_bytes() == 0; }, 60.0);
    delete w;
    std::_Exit(0);
  }
  Ring* r = nullptr;
  dgi_shm::wait_until([&] { return (r = Ring::try_open(name)) != nullptr; }, 60.0);
  if (r == nullptr) fail("fork", "ring never created");
  shm_unlink(name.c_str());
  consume("fork", r, n, max_len);
  int st = 0;
  waitpid(pid, &st, 0);
  if (!WIFEXITED(st) || WEXITSTATUS(st) != 0) fail("fork", "producer exited with " + std::to_string(st));
  delete r;
  std::printf("ok fork %llu\n", static_cast<unsigned long long>(n));
  return 0;
}

int run_limits() {
  const std::string name = ring_name("lim");
  Ring* w = Ring::create(name, 4096);
  Ring* r = Ring::try_open(name);
  shm_unlink(name.c_str());
  if (r == nullptr) fail("limits", "open");
  const std::string a(1000, 'a'), b(1000, 'b'), c(1000, 'c'), d(1000, 'd'), big(1500, 'x');
  if (!w->try_write(a.data(), a.size()) || !w->try_write(b.data(), b.size()) || !w->try_write(c.data(), c.size()))
    fail("limits", "three 1000-byte messages must fit 4096");
  if (w->try_write(big.data(), big.size())) fail("limits", "full ring accepted a message");
  if (w->write(big.data(), big.size(), 0.05)) fail("limits", "blocking write on a full ring must time out");
  if (r->read_one() != a) fail("limits", "a");
  if (!w->try_write(d.data(), d.size())) fail("limits", "room after a read");   // wraps around the end
  if (r->read_one() != b || r->read_one() != c || r->read_one() != d) fail("limits", "order after wrap");
  bool threw = false;
  try {
    const std::string huge(3000, 'h');
    w->try_write(huge.data(), huge.size());
  } catch (const std::length_error&) {
    threw = true;
  }
  if (!threw) fail("limits", "oversize message accepted");
  // exact fill to the end of the data area, then a message that starts at offset 0
  for (int k = 0; k < 64; ++k) {
    const std::string m = make_msg(static_cast<uint64_t>(k), 1900);
    if (!w->write(m.data(), m.size(), 1.0)) fail("limits", "write");
    check("limits", static_cast<uint64_t>(k), r->read_one(), 1900);
  }
  if (r->has_message()) fail("limits", "empty ring reports a message");
  delete r;
  delete w;
  std::printf("ok limits 68\n");
  return 0;
}

}  // namespace

int main(int argc, char** argv) {
  const std::string mode = argc > 1 ? argv[1] : "all";
  const uint64_t n = argc > 2 ? std::strtoull(argv[2], nullptr, 10) : 20000;
  try {
    if (mode == "threads" || mode == "all") run_threads(n);
    if (mode == "fork" || mode == "all") run_fork(n);
    if (mode == "limits" || mode == "all") run_limits();
  } catch (const std::exception& e) {
    fail(mode.c_str(), e.what());
  }
  return 0;
}
