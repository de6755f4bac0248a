// ADAPT host runtime (C++17): framing transport + codecs.
#pragma once
#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

namespace adapt_rt {

// ---- xxHash32 / LZ4 (lz4.cpp)
uint32_t xxh32(const uint8_t* p, size_t len, uint32_t seed);
size_t lz4_block_bound(size_t n);
size_t lz4_block_compress(const uint8_t* src, size_t n, uint8_t* dst, size_t cap, int accel);
size_t lz4_block_decompress(const uint8_t* src, size_t n, uint8_t* dst, size_t cap);
std::vector<uint8_t> lz4_frame_compress(const uint8_t* src, size_t n, int accel);
std::vector<uint8_t> lz4_frame_decompress(const uint8_t* src, size_t n);

// ---- reversible zfp-style codec (zfp_rev.cpp)
struct ZfpHeader {
  int dtype;                  // 0 = float32, 1 = float64
  std::vector<size_t> shape;  // C order
  size_t payload_off;
};
std::vector<uint8_t> zfp_compress(const void* src, int dtype_code, const std::vector<size_t>& shape, int threads);
ZfpHeader zfp_header(const uint8_t* data, size_t n);
void zfp_decompress(const uint8_t* data, size_t n, void* dst, int threads);

// ---- framing transport (framing.cpp): 8-byte big-endian length + body
// Works on blocking and non-blocking sockets (poll() on EAGAIN).
// recv_frame returns false on a clean EOF before any header byte.
void send_all(int fd, const uint8_t* p, size_t n, size_t chunk, int timeout_ms);
void send_frame(int fd, const uint8_t* p, size_t n, size_t chunk, int timeout_ms);
bool recv_exact(int fd, uint8_t* p, size_t n, size_t chunk, int timeout_ms, bool eof_ok_at_start);
bool recv_frame(int fd, std::vector<uint8_t>& out, size_t chunk, int timeout_ms, size_t max_len);

}  // namespace adapt_rt
