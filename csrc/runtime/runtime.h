// ADAPT host runtime (C++17): framing transport + codecs.
#pragma once
#include <cstddef>
#include <cstdint>
#include <string>
#include <utility>
#include <tuple>
#include <vector>

namespace adapt_rt {

// ---- xxHash32 / LZ4 (lz4.cpp)
uint32_t xxh32(const uint8_t* p, size_t len, uint32_t seed);
size_t lz4_block_bound(size_t n);
size_t lz4_block_compress(const uint8_t* src, size_t n, uint8_t* dst, size_t cap, int accel);
size_t lz4_block_decompress(const uint8_t* src, size_t n, uint8_t* dst, size_t cap);
std::vector<uint8_t> lz4_frame_compress(const uint8_t* src, size_t n, int accel);
std::vector<uint8_t> lz4_frame_decompress(const uint8_t* src, size_t n);
struct Lz4FrameBlocks {
  uint64_t content_size;
  size_t block_max;
  bool independent;
  std::vector<uint32_t> offsets;   // payload offset of each block within the frame
  std::vector<uint32_t> words;     // block size words (high bit = stored raw)
};
Lz4FrameBlocks lz4_frame_blocks(const uint8_t* src, size_t n);

// ---- zero-value compression stream "AZVC" (zvc.cpp; GPU twin: kernels/zvc_gpu.hip)
struct ZvcHeader {
  uint64_t n;
  int esz;
  uint32_t nseg;
  std::vector<uint32_t> offsets;   // segment offsets relative to the payload start
};
std::vector<uint8_t> zvc_compress(const uint8_t* in, size_t n, int esz);
ZvcHeader zvc_header(const uint8_t* p, size_t len);
void zvc_decompress(const uint8_t* p, size_t len, uint8_t* out);

// ---- reversible zfp-style codec (zfp_rev.cpp)
struct ZfpHeader {
  int dtype;                  // 0 = float32, 1 = float64
  std::vector<size_t> shape;  // C order
  size_t payload_off;
  size_t chunk_blocks;        // blocks per independently coded chunk (v1: 4096)
};
// chunk_blocks 0 / 4096: version-1 container; any other value: version 2 (header carries it)
std::vector<uint8_t> zfp_compress(const void* src, int dtype_code, const std::vector<size_t>& shape, int threads,
                                  size_t chunk_blocks = 0);
ZfpHeader zfp_header(const uint8_t* data, size_t n);
void zfp_decompress(const uint8_t* data, size_t n, void* dst, int threads);

// ---- framing transport (framing.cpp): 8-byte big-endian length + body
// Works on blocking and non-blocking sockets (poll() on EAGAIN).
// recv_frame returns false on a clean EOF before any header byte.
void send_all(int fd, const uint8_t* p, size_t n, size_t chunk, int timeout_ms);
void send_frame(int fd, const uint8_t* p, size_t n, size_t chunk, int timeout_ms);
// one frame whose body is the concatenation of `parts` (no staging copy)
void send_frame_parts(int fd, const std::vector<std::pair<const uint8_t*, size_t>>& parts, size_t chunk,
                      int timeout_ms);
bool recv_exact(int fd, uint8_t* p, size_t n, size_t chunk, int timeout_ms, bool eof_ok_at_start);
bool recv_frame(int fd, std::vector<uint8_t>& out, size_t chunk, int timeout_ms, size_t max_len);

// ---- liveness heartbeats over UDP (heartbeat.cpp): GIL-free sender / monitor threads
void* hb_sender_start(const std::string& host, int port, const std::string& id, int period_us);
void hb_sender_stop(void* h);
// completed-micro-batch counter of `epoch` and measured seconds-per-micro-batch (ns, 0 = keep), carried by
// every beat
void hb_sender_progress(void* h, uint64_t value, uint64_t stage_ns, uint64_t epoch);
// id -> (progress counter, seconds since it last changed, reported seconds per micro-batch, epoch)
std::vector<std::tuple<std::string, uint64_t, double, double, uint64_t>> hb_monitor_progress(void* h);
void* hb_monitor_start(int port);
int hb_monitor_port(void* h);
std::vector<std::pair<std::string, double>> hb_monitor_ages(void* h);   // id -> seconds since its last beat
void hb_monitor_forget(void* h, const std::string& id);
void hb_monitor_stop(void* h);

// ---- bulk host copy split over threads (framing.cpp)
void parallel_copy(uint8_t* dst, const uint8_t* src, size_t n, int threads);

}  // namespace adapt_rt
