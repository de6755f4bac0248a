// Framed socket transport, wire-compatible with the reference's
// `socket_send` / `socket_recv` (`src/node_state.py:39-161`):
//
//   frame := u64 big-endian body length || body
//
// The body is written / read in `chunk`-sized system calls; on EAGAIN /
// EWOULDBLOCK the call waits with poll() (the reference busy-waits with
// select()).  A clean EOF before the first header byte is reported as "no
// frame" (the reference returns b''); EOF anywhere later raises, as do
// timeouts.  All calls run without the GIL (bindings.cpp).
#include <errno.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <chrono>
#include <cstring>
#include <stdexcept>
#include <string>

#include "runtime.h"

#include <algorithm>
#include <cstring>
#include <thread>
#include <vector>

namespace adapt_rt {

static void wait_fd(int fd, short ev, int timeout_ms) {
  struct pollfd p;
  p.fd = fd;
  p.events = ev;
  p.revents = 0;
  for (;;) {
    int r = poll(&p, 1, timeout_ms < 0 ? -1 : timeout_ms);
    if (r > 0) return;
    if (r == 0) throw std::runtime_error("socket timeout");
    if (errno == EINTR) continue;
    throw std::runtime_error(std::string("poll: ") + strerror(errno));
  }
}

void send_all(int fd, const uint8_t* p, size_t n, size_t chunk, int timeout_ms) {
  if (chunk == 0) chunk = n ? n : 1;
  size_t off = 0;
  while (off < n) {
    size_t want = n - off < chunk ? n - off : chunk;
    ssize_t s = ::send(fd, p + off, want, MSG_NOSIGNAL);
    if (s > 0) {
      off += (size_t)s;
      continue;
    }
    if (s < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) {
      wait_fd(fd, POLLOUT, timeout_ms);
      continue;
    }
    if (s < 0 && errno == EINTR) continue;
    throw std::runtime_error(std::string("send: ") + (s < 0 ? strerror(errno) : "connection closed"));
  }
}

void send_frame(int fd, const uint8_t* p, size_t n, size_t chunk, int timeout_ms) {
  uint8_t hdr[8];
  uint64_t v = n;
  for (int i = 7; i >= 0; --i) {
    hdr[i] = (uint8_t)(v & 0xFF);
    v >>= 8;
  }
  send_all(fd, hdr, 8, 8, timeout_ms);
  send_all(fd, p, n, chunk, timeout_ms);
}

void send_frame_parts(int fd, const std::vector<std::pair<const uint8_t*, size_t>>& parts, size_t chunk,
                      int timeout_ms) {
  uint64_t v = 0;
  for (auto& pr : parts) v += pr.second;
  uint8_t hdr[8];
  for (int i = 7; i >= 0; --i) {
    hdr[i] = (uint8_t)(v & 0xFF);
    v >>= 8;
  }
  send_all(fd, hdr, 8, 8, timeout_ms);
  for (auto& pr : parts) send_all(fd, pr.first, pr.second, chunk, timeout_ms);
}

bool recv_exact(int fd, uint8_t* p, size_t n, size_t chunk, int timeout_ms, bool eof_ok_at_start) {
  if (chunk == 0) chunk = n ? n : 1;
  size_t off = 0;
  while (off < n) {
    size_t want = n - off < chunk ? n - off : chunk;
    ssize_t r = ::recv(fd, p + off, want, 0);
    if (r > 0) {
      off += (size_t)r;
      continue;
    }
    if (r == 0) {
      if (off == 0 && eof_ok_at_start) return false;
      throw std::runtime_error("connection closed mid-frame");
    }
    if (errno == EAGAIN || errno == EWOULDBLOCK) {
      wait_fd(fd, POLLIN, timeout_ms);
      continue;
    }
    if (errno == EINTR) continue;
    throw std::runtime_error(std::string("recv: ") + strerror(errno));
  }
  return true;
}

bool recv_frame(int fd, std::vector<uint8_t>& out, size_t chunk, int timeout_ms, size_t max_len) {
  uint8_t hdr[8];
  if (!recv_exact(fd, hdr, 8, 8, timeout_ms, true)) return false;
  uint64_t n = 0;
  for (int i = 0; i < 8; ++i) n = (n << 8) | hdr[i];
  if (max_len && n > max_len) throw std::runtime_error("frame larger than max_len");
  out.resize((size_t)n);
  if (n) recv_exact(fd, out.data(), (size_t)n, chunk, timeout_ms, false);
  return true;
}

// Large request copies (a bs=32 fp32 batch is 19 MB) into shared-memory slots:
// one thread's memcpy runs at ~10 GB/s, a few threads on disjoint 64-byte-aligned
// ranges reach the socket's memory bandwidth.  Below 1 MB a plain memcpy.
void parallel_copy(uint8_t* dst, const uint8_t* src, size_t n, int threads) {
  if (threads <= 1 || n < (size_t(1) << 20)) {
    std::memcpy(dst, src, n);
    return;
  }
  if (threads > 16) threads = 16;
  const size_t per = (((n + threads - 1) / threads) + 63) & ~size_t(63);
  std::vector<std::thread> pool;
  pool.reserve(threads - 1);
  for (int t = 1; t < threads; ++t) {
    const size_t b = per * t;
    if (b >= n) break;
    const size_t len = std::min(per, n - b);
    pool.emplace_back([=] { std::memcpy(dst + b, src + b, len); });
  }
  std::memcpy(dst, src, std::min(per, n));
  for (auto& th : pool) th.join();
}

}  // namespace adapt_rt
