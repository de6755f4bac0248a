// Standalone self-test of the host runtime, built under sanitizers
// (tools/sanitize.sh: ASan+UBSan and TSan).  Exercises every codec on random
// and adversarial inputs, rejects corrupted streams without reading out of
// bounds, and runs the framing transport over a socketpair with a concurrent
// sender thread (the data plane's threading pattern).
#include <sys/socket.h>
#include <unistd.h>

#include <cstdio>
#include <cstring>
#include <random>
#include <stdexcept>
#include <thread>
#include <vector>

#include "runtime.h"

using namespace adapt_rt;

static int failures = 0;
#define CHECK(c)                                                   \
  do {                                                             \
    if (!(c)) {                                                    \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++failures;                                                  \
    }                                                              \
  } while (0)

static std::vector<uint8_t> rand_bytes(std::mt19937& g, size_t n, int alphabet) {
  std::vector<uint8_t> v(n);
  std::uniform_int_distribution<int> d(0, alphabet - 1);
  for (auto& b : v) b = (uint8_t)d(g);
  return v;
}

int main() {
  std::mt19937 g(1234);
  // ---- LZ4 frame
  for (size_t n : {0ul, 1ul, 11ul, 12ul, 13ul, 300ul, 65536ul, 300001ul}) {
    for (int alpha : {2, 256}) {
      auto src = rand_bytes(g, n, alpha);
      auto fr = lz4_frame_compress(src.data(), src.size(), 1);
      auto back = lz4_frame_decompress(fr.data(), fr.size());
      CHECK(back == src);
      // truncations and bit flips must throw, never crash
      for (size_t cut : {fr.size() / 2, fr.size() - 1}) {
        if (cut == 0) continue;
        try {
          lz4_frame_decompress(fr.data(), cut);
          CHECK(false);
        } catch (const std::exception&) {
        }
      }
      if (fr.size() > 20) {
        auto bad = fr;
        bad[fr.size() / 2] ^= 0x5A;
        try {
          auto r = lz4_frame_decompress(bad.data(), bad.size());
          (void)r;   // may decode to garbage only if the checksum also matched (it must not)
          CHECK(false);
        } catch (const std::exception&) {
        }
      }
    }
  }
  // ---- zfp reversible
  {
    std::normal_distribution<float> nd(0.f, 3.f);
    for (auto shape : std::vector<std::vector<size_t>>{{1}, {5}, {3, 7}, {4, 5, 6}, {2, 3, 9, 17}}) {
      size_t n = 1;
      for (auto s : shape) n *= s;
      std::vector<float> a(n);
      for (auto& x : a) x = nd(g);
      auto c = zfp_compress(a.data(), 0, shape, 3);
      std::vector<float> b(n);
      zfp_decompress(c.data(), c.size(), b.data(), 3);
      CHECK(std::memcmp(a.data(), b.data(), n * 4) == 0);
      try {
        zfp_decompress(c.data(), c.size() / 2, b.data(), 2);
        CHECK(false);
      } catch (const std::exception&) {
      }
    }
  }
  // ---- zvc
  for (size_t n : {1ul, 63ul, 4096ul, 9001ul}) {
    auto src = rand_bytes(g, n * 2, 4);   // many zero bytes
    auto s = zvc_compress(src.data(), n, 2);
    std::vector<uint8_t> back(n * 2);
    zvc_decompress(s.data(), s.size(), back.data());
    CHECK(back == src);
    try {
      zvc_decompress(s.data(), s.size() - 1, back.data());
      CHECK(false);
    } catch (const std::exception&) {
    }
  }
  // ---- framing with a concurrent sender (blocking sockets)
  {
    int sv[2];
    CHECK(socketpair(AF_UNIX, SOCK_STREAM, 0, sv) == 0);
    auto payload = rand_bytes(g, 3 << 20, 256);
    std::thread tx([&] {
      for (int i = 0; i < 3; ++i) send_frame(sv[0], payload.data(), payload.size(), 512000, 10000);
      send_frame(sv[0], payload.data(), 0, 512000, 10000);
      ::shutdown(sv[0], SHUT_WR);
    });
    std::vector<uint8_t> got;
    for (int i = 0; i < 3; ++i) {
      CHECK(recv_frame(sv[1], got, 4096, 10000, 0));
      CHECK(got == payload);
    }
    CHECK(recv_frame(sv[1], got, 4096, 10000, 0) && got.empty());
    CHECK(!recv_frame(sv[1], got, 4096, 10000, 0));   // clean EOF
    tx.join();
    close(sv[0]);
    close(sv[1]);
  }
  std::printf("selftest %s (%d failures)\n", failures ? "FAILED" : "passed", failures);
  return failures ? 1 : 0;
}
