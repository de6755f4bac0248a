// GPU LZ4 codec for activations (gfx950), producing / consuming STANDARD LZ4
// frames so a GPU-compressed activation can be decoded by any LZ4 frame
// decoder (our host codec in csrc/runtime/lz4.cpp, python-lz4, lz4 CLI).
//
// The reference compresses every activation on the CPU before each TCP hop
// (`src/node.py:178`, `src/dispatcher.py:92-98`).  Here compression runs on a
// side HIP stream right after the producing slice, overlapped with the next
// micro-batch's compute (codec/gpu_lz4.py, codec/wire.py, parallel/pipeline.py).
//
// Layout: the input is cut into CHUNK-byte chunks; each chunk is one
// independent LZ4 block (frame FLG: independent blocks, content size, no
// checksums; BD: 64 KiB max block).  Incompressible chunks are stored raw
// (block size high bit).
//
// v2 (wave-parallel; v1 ran one THREAD per 1 KiB chunk with a serial byte
// matcher and measured 1.3-5 GB/s, profiles/codec_bench_r50_bs32.json):
//
// * encode: one 64-lane wave per 2 KiB chunk staged in LDS.  Hashing is
//   data-parallel: 64 consecutive positions per step read the wave-private
//   hash table (positions of EARLIER steps), verify their 4-byte candidate,
//   publish a ballot bitmask of match starts, then insert themselves.  The
//   greedy parse is a wave-uniform walk over that bitmask (ctz per 64
//   positions); match extension compares 64 bytes per step (ballot of the
//   first mismatch) and literal copies are lane-parallel.  Incompressible
//   data costs one hashing pass plus a raw copy.
// * a single workgroup prefix-sums the block sizes; a pack kernel (one wave
//   per block) scatters the blocks after the 15-byte frame header.
// * decode: one wave per block; the compressed block is staged in LDS, the
//   sequence headers are read wave-uniformly and literals / matches are
//   copied lane-parallel (overlapping matches in rounds of `offset` bytes),
//   then the chunk leaves LDS in 16-byte stores.  Block offsets come either
//   from the host frame parser or, for device-to-device links, from the
//   same scan over the block-size table (lz4_gpu_decompress_dev).
#include "kernels.h"

namespace adapt {

namespace {
constexpr int CHUNK = 2048;                          // bytes per LZ4 block
constexpr int BOUND = 2080;                          // >= CHUNK + CHUNK/255 + 16, multiple of 16
constexpr int HBITS = 11;
constexpr int WAVES = 4;                             // chunks (waves) per workgroup
constexpr int MINMATCH = 4, LASTLIT = 5, MFLIMIT = 12;
constexpr int HDR = 15;                              // frame header bytes (magic, FLG, BD, size, HC)

struct __attribute__((aligned(16))) EncLds {
  uint32_t data[CHUNK / 4 + 4];                      // chunk + 16 zero bytes
  uint16_t refs[CHUNK];                              // hash candidate of each position
  uint16_t tab[1 << HBITS];                          // hash table; reused as the output buffer (4 KiB)
  uint64_t mask[CHUNK / 64];                         // verified match starts
};
static_assert(sizeof(uint16_t) * (1 << HBITS) >= CHUNK + 64, "output buffer");

struct __attribute__((aligned(16))) DecLds {
  uint8_t cbuf[BOUND + 16];
  uint8_t obuf[CHUNK];
};

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ uint32_t lds32(const uint32_t* d, int p) {
  const uint32_t lo = d[p >> 2], hi = d[(p >> 2) + 1];
  return __builtin_amdgcn_alignbyte(hi, lo, (uint32_t)(p & 3));
}
__device__ __forceinline__ uint32_t hsh(uint32_t v) { return (v * 2654435761u) >> (32 - HBITS); }

// lane-parallel LZ4 length continuation: len / 255 bytes of 255, then the remainder
__device__ __forceinline__ int put_len(uint8_t* o, int len, int lane) {
  const int nb = len / 255 + 1;
  for (int j = lane; j < nb; j += 64) o[j] = (uint8_t)(j < nb - 1 ? 255 : len - 255 * (nb - 1));
  return nb;
}
}  // namespace

// scratch[c * BOUND ...] <- compressed chunk c; sizes[c] = LZ4 block-size word
__global__ __launch_bounds__(WAVES * 64) void lz4_enc_chunks(const uint8_t* __restrict__ in, size_t n,
                                                             uint8_t* __restrict__ scratch,
                                                             uint32_t* __restrict__ sizes, int nchunks) {
  __shared__ EncLds lds_all[WAVES];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int c = blockIdx.x * WAVES + wave;
  if (c >= nchunks) return;                          // waves are independent: no block barrier below
  EncLds& L = lds_all[wave];
  uint8_t* data8 = (uint8_t*)L.data;
  const size_t base = (size_t)c * CHUNK;
  const int len = (int)min((size_t)CHUNK, n - base);
  const uint8_t* src = in + base;

  // ---- stage the chunk (16-byte loads when whole and aligned)
  if (len == CHUNK && (((uintptr_t)src) & 15) == 0) {
    const u32x4* s4 = (const u32x4*)src;
    const u32x4 v0 = s4[lane], v1 = s4[lane + 64];
    ((u32x4*)L.data)[lane] = v0;
    ((u32x4*)L.data)[lane + 64] = v1;
    if (lane < 4) L.data[CHUNK / 4 + lane] = 0;
  } else {
    for (int k = lane; k < CHUNK + 16; k += 64) data8[k] = k < len ? src[k] : (uint8_t)0;
  }
  {
    u32x4* t4 = (u32x4*)L.tab;
    const u32x4 ones = (u32x4){0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
    for (int k = lane; k < (1 << HBITS) * 2 / 16; k += 64) t4[k] = ones;
  }
  wave_sync();

  // ---- hashing: 64 positions per step against the table of earlier steps
  const int mflimit = len - MFLIMIT;                 // match starts p in [1, mflimit)
  const int nwords = mflimit > 0 ? (mflimit + 63) >> 6 : 0;
  for (int b = 0; b < nwords; ++b) {
    const int p = b * 64 + lane;
    const bool inr = p < mflimit;
    const uint32_t seq = lds32(L.data, p);
    const uint32_t h = hsh(seq);
    const uint32_t cand = inr ? L.tab[h] : 0xFFFFu;
    const bool ok = inr && p >= 1 && cand != 0xFFFFu && lds32(L.data, (int)cand) == seq;
    const uint64_t m = __ballot(ok);
    if (lane == 0) L.mask[b] = m;
    L.refs[p] = (uint16_t)cand;
    wave_sync();
    if (inr) L.tab[h] = (uint16_t)p;                 // the highest lane of a collision wins
    wave_sync();
  }

  // ---- greedy parse over the match-start bitmask (wave-uniform control flow)
  uint8_t* out = (uint8_t*)L.tab;
  int anchor = 0, ip = 0, op = 0;
  bool raw = false;
  for (;;) {
    int p = -1;
    for (int w = ip >> 6; w < nwords; ++w) {
      uint64_t m = L.mask[w];
      if (w == (ip >> 6)) m &= ~0ull << (ip & 63);
      if (m) {
        p = (w << 6) + __builtin_ctzll(m);
        break;
      }
    }
    if (p < 0) break;
    const int ref = L.refs[p];
    const int maxl = (len - LASTLIT) - p;            // longest legal match here (> MINMATCH)
    int ml = MINMATCH;
    for (;;) {
      const int k = ml + lane;
      const bool stop = k >= maxl || data8[p + k] != data8[ref + k];
      const uint64_t bm = __ballot(stop);
      if (bm) {
        ml += __builtin_ctzll(bm);
        break;
      }
      ml += 64;
    }
    const int lit = p - anchor;
    const int mlc = ml - MINMATCH;
    const int need = 1 + (lit >= 15 ? (lit - 15) / 255 + 1 : 0) + lit + 2 + (mlc >= 15 ? (mlc - 15) / 255 + 1 : 0);
    if (op + need + 1 > len) {                       // could only expand: store the chunk raw
      raw = true;
      break;
    }
    int o = op;
    if (lane == 0) out[o] = (uint8_t)(((lit >= 15 ? 15 : lit) << 4) | (mlc >= 15 ? 15 : mlc));
    ++o;
    if (lit >= 15) o += put_len(out + o, lit - 15, lane);
    for (int k = lane; k < lit; k += 64) out[o + k] = data8[anchor + k];
    o += lit;
    const int off = p - ref;
    if (lane == 0) {
      out[o] = (uint8_t)(off & 0xFF);
      out[o + 1] = (uint8_t)(off >> 8);
    }
    o += 2;
    if (mlc >= 15) o += put_len(out + o, mlc - 15, lane);
    op = o;
    anchor = ip = p + ml;
  }
  if (!raw) {                                        // last literals
    const int lit = len - anchor;
    const int need = 1 + (lit >= 15 ? (lit - 15) / 255 + 1 : 0) + lit;
    if (op + need >= len) {
      raw = true;
    } else {
      int o = op;
      if (lane == 0) out[o] = (uint8_t)((lit >= 15 ? 15 : lit) << 4);
      ++o;
      if (lit >= 15) o += put_len(out + o, lit - 15, lane);
      for (int k = lane; k < lit; k += 64) out[o + k] = data8[anchor + k];
      op = o + lit;
    }
  }
  if (raw) {
    if (lane == 0) sizes[c] = (uint32_t)len | 0x80000000u;
    return;
  }
  wave_sync();
  u32x4* dst = (u32x4*)(scratch + (size_t)c * BOUND);
  const u32x4* o4 = (const u32x4*)out;
  for (int v = lane; v < (op + 15) >> 4; v += 64) dst[v] = o4[v];
  if (lane == 0) sizes[c] = (uint32_t)op;
}

// single-workgroup exclusive scan of (4 + payload) over the blocks -> offsets
// (relative to the first block header); frame bytes in *total (if given)
__global__ __launch_bounds__(1024) void lz4_scan(const uint32_t* __restrict__ sizes, uint32_t* __restrict__ offs,
                                                 int nchunks, uint64_t* __restrict__ total) {
  __shared__ uint32_t part[1024];
  const int t = threadIdx.x;
  const int per = (nchunks + 1023) / 1024;
  const int b0 = t * per, b1 = min(nchunks, b0 + per);
  uint32_t s = 0;
  for (int i = b0; i < b1; ++i) s += 4 + (sizes[i] & 0x7FFFFFFFu);
  part[t] = s;
  __syncthreads();
  for (int d = 1; d < 1024; d <<= 1) {        // Hillis-Steele inclusive scan
    uint32_t v = t >= d ? part[t - d] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  uint32_t run = t ? part[t - 1] : 0;
  for (int i = b0; i < b1; ++i) {
    offs[i] = run;
    run += 4 + (sizes[i] & 0x7FFFFFFFu);
  }
  if (t == 1023 && total) *total = (uint64_t)HDR + part[1023] + 4;   // header + blocks + end mark
}

// one wave per block: size word + payload at frame + HDR + offs[c]
__global__ __launch_bounds__(WAVES * 64) void lz4_pack(const uint8_t* __restrict__ in, size_t n,
                                                       const uint8_t* __restrict__ scratch,
                                                       const uint32_t* __restrict__ sizes,
                                                       const uint32_t* __restrict__ offs, int nchunks,
                                                       uint8_t* __restrict__ out, const uint64_t* total) {
  const int lane = threadIdx.x & 63;
  const int c = blockIdx.x * WAVES + (threadIdx.x >> 6);
  if (c == 0 && lane == 0) {
    // frame header: magic, FLG (v01, B.Indep, C.Size), BD (64 KiB), content size, HC
    uint8_t h[HDR] = {0x04, 0x22, 0x4D, 0x18, (1u << 6) | (1u << 5) | (1u << 3), 4u << 4};
    uint64_t cs = n;
    for (int i = 0; i < 8; ++i) h[6 + i] = (uint8_t)(cs >> (8 * i));
    // xxh32(h+4, 10, 0) >> 8 & 0xFF computed inline
    const uint32_t P1 = 2654435761U, P2 = 2246822519U, P3 = 3266489917U, P4 = 668265263U, P5 = 374761393U;
    uint32_t acc = P5 + 10u;
    const uint8_t* q = h + 4;
    for (int i = 0; i < 2; ++i) {
      uint32_t v = (uint32_t)q[4 * i] | ((uint32_t)q[4 * i + 1] << 8) | ((uint32_t)q[4 * i + 2] << 16) |
                   ((uint32_t)q[4 * i + 3] << 24);
      acc += v * P3;
      acc = ((acc << 17) | (acc >> 15)) * P4;
    }
    for (int i = 8; i < 10; ++i) {
      acc += q[i] * P5;
      acc = ((acc << 11) | (acc >> 21)) * P1;
    }
    acc ^= acc >> 15; acc *= P2; acc ^= acc >> 13; acc *= P3; acc ^= acc >> 16;
    h[14] = (uint8_t)((acc >> 8) & 0xFF);
    for (int i = 0; i < HDR; ++i) out[i] = h[i];
    const uint64_t tot = *total;
    for (int i = 0; i < 4; ++i) out[tot - 4 + i] = 0;   // end mark
  }
  if (c >= nchunks) return;
  const uint32_t w = sizes[c];
  uint8_t* o = out + HDR + offs[c];
  if (lane < 4) o[lane] = (uint8_t)(w >> (8 * lane));
  const uint32_t len = w & 0x7FFFFFFFu;
  const uint8_t* src = (w & 0x80000000u) ? in + (size_t)c * CHUNK : scratch + (size_t)c * BOUND;
  for (uint32_t i = lane; i < len; i += 64) o[4 + i] = src[i];
}

// one wave per block: decode block c (payload at frame + offs[c] + bias, size word
// sizes[c]) into out + c*CHUNK
__global__ __launch_bounds__(WAVES * 64) void lz4_dec_chunks(const uint8_t* __restrict__ frame,
                                                             const uint32_t* __restrict__ offs,
                                                             const uint32_t* __restrict__ sizes, int nchunks,
                                                             int bias, uint8_t* __restrict__ out, size_t n,
                                                             int* __restrict__ err) {
  __shared__ DecLds lds_all[WAVES];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int c = blockIdx.x * WAVES + wave;
  if (c >= nchunks) return;
  DecLds& L = lds_all[wave];
  const uint32_t w = sizes[c];
  const int len = (int)(w & 0x7FFFFFFFu);
  const uint8_t* ip0 = frame + offs[c] + bias;
  const int cap = (int)min((size_t)CHUNK, n - (size_t)c * CHUNK);
  uint8_t* dst = out + (size_t)c * CHUNK;
  if (w & 0x80000000u) {
    if (len != cap) {
      if (lane == 0) atomicOr(err, 1);
      return;
    }
    for (int k = lane; k < len; k += 64) L.obuf[k] = ip0[k];
  } else {
    if (len > BOUND) {
      if (lane == 0) atomicOr(err, 2);
      return;
    }
    for (int k = lane; k < len; k += 64) L.cbuf[k] = ip0[k];
    wave_sync();
    const uint8_t* cb = L.cbuf;
    int ip = 0, o = 0, bad = 0;
    while (ip < len) {
      const int token = cb[ip++];
      int lit = token >> 4;
      if (lit == 15) {
        int b;
        do { b = cb[ip++]; lit += b; } while (b == 255 && ip < len);
      }
      if (o + lit > cap || ip + lit > len) { bad = 2; break; }
      for (int k = lane; k < lit; k += 64) L.obuf[o + k] = cb[ip + k];
      o += lit;
      ip += lit;
      if (ip >= len) break;
      const int off = cb[ip] | (cb[ip + 1] << 8);
      ip += 2;
      int ml = token & 15;
      if (ml == 15) {
        int b;
        do { b = cb[ip++]; ml += b; } while (b == 255 && ip < len);
      }
      ml += MINMATCH;
      if (off == 0 || off > o || o + ml > cap) { bad = 4; break; }
      wave_sync();
      const int step = off < 64 ? off : 64;         // an overlapping match copies `off` bytes per round
      for (int d = 0; d < ml; d += step) {
        const int k = d + lane;
        if (lane < step && k < ml) L.obuf[o + k] = L.obuf[o - off + k];
        wave_sync();
      }
      o += ml;
    }
    if (!bad && o != cap) bad = 8;
    if (bad) {
      if (lane == 0) atomicOr(err, bad);
      return;
    }
  }
  wave_sync();
  if (cap == CHUNK && (((uintptr_t)dst) & 15) == 0) {
    u32x4* d4 = (u32x4*)dst;
    const u32x4* s4 = (const u32x4*)L.obuf;
    d4[lane] = s4[lane];
    d4[lane + 64] = s4[lane + 64];
  } else {
    for (int k = lane; k < cap; k += 64) dst[k] = L.obuf[k];
  }
}

// ---------------------------------------------------------------- launchers
int lz4_gpu_chunk() { return CHUNK; }
size_t lz4_gpu_scratch_bytes(size_t n) {
  const size_t nch = (n + CHUNK - 1) / CHUNK;
  return nch * BOUND;
}
size_t lz4_gpu_max_frame(size_t n) {
  const size_t nch = (n + CHUNK - 1) / CHUNK;
  return HDR + nch * (4 + CHUNK) + 4;
}

// sizes/offs: >= nchunks u32 each; total: one u64 (frame bytes)
hipError_t lz4_gpu_compress(const uint8_t* in, size_t n, uint8_t* scratch, uint32_t* sizes, uint32_t* offs,
                            uint8_t* out, uint64_t* total, hipStream_t s) {
  const int nch = (int)((n + CHUNK - 1) / CHUNK);
  if (nch == 0 || n > 0xFFFFFFFFull - (size_t)nch * 8) return hipErrorInvalidValue;
  const int grid = (nch + WAVES - 1) / WAVES;
  hipLaunchKernelGGL(lz4_enc_chunks, dim3(grid), dim3(WAVES * 64), 0, s, in, n, scratch, sizes, nch);
  hipLaunchKernelGGL(lz4_scan, dim3(1), dim3(1024), 0, s, sizes, offs, nch, total);
  hipLaunchKernelGGL(lz4_pack, dim3(grid), dim3(WAVES * 64), 0, s, in, n, scratch, sizes, offs, nch, out, total);
  return hipGetLastError();
}

// offs = payload offsets within the frame (host frame parser)
hipError_t lz4_gpu_decompress(const uint8_t* frame, const uint32_t* offs, const uint32_t* sizes, int nchunks,
                              uint8_t* out, size_t n, int* err, hipStream_t s) {
  if (nchunks < 1 || (size_t)nchunks != (n + CHUNK - 1) / CHUNK) return hipErrorInvalidValue;
  hipLaunchKernelGGL(lz4_dec_chunks, dim3((nchunks + WAVES - 1) / WAVES), dim3(WAVES * 64), 0, s, frame, offs, sizes,
                     nchunks, 0, out, n, err);
  return hipGetLastError();
}

// device-resident frame + its block-size table (e.g. both received over RCCL):
// offsets come from the encoder's scan, no host round trip
hipError_t lz4_gpu_decompress_dev(const uint8_t* frame, const uint32_t* sizes, int nchunks, uint32_t* offs_scratch,
                                  uint8_t* out, size_t n, int* err, hipStream_t s) {
  if (nchunks < 1 || (size_t)nchunks != (n + CHUNK - 1) / CHUNK) return hipErrorInvalidValue;
  hipLaunchKernelGGL(lz4_scan, dim3(1), dim3(1024), 0, s, sizes, offs_scratch, nchunks, (uint64_t*)nullptr);
  hipLaunchKernelGGL(lz4_dec_chunks, dim3((nchunks + WAVES - 1) / WAVES), dim3(WAVES * 64), 0, s, frame,
                     (const uint32_t*)offs_scratch, sizes, nchunks, HDR + 4, out, n, err);
  return hipGetLastError();
}

}  // namespace adapt
