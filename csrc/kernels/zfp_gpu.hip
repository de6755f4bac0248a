// GPU reversible zfp-style codec for float32 arrays, bit-exact with the host
// codec (csrc/runtime/zfp_rev.cpp) in its version-2 container with
// chunk_blocks = 1.
//
// The reference compresses every hop with zfp (reversible) + LZ4 on the CPU
// (`src/dispatcher.py:92-98`, `src/node.py:122-125`); here the block
// transform runs on a side HIP stream.  Per 4^d block (one thread each):
// gather with edge replication -> order-preserving integers -> reversible
// lifting along every axis -> total-sequency order -> negabinary -> embedded
// bit-plane coding with group tests, into a word-aligned private stream.  A
// single-workgroup scan turns the per-block word counts into offsets and a
// pack kernel concatenates the streams after the word-count table, which is
// exactly the host container's chunk table + payload.  Decoding is the same
// in reverse, again one block per thread.
#include "kernels.h"

namespace adapt {

namespace {

struct ZGeom {
  int d;
  uint32_t shape[4];   // axis 0 fastest (C order reversed)
  uint32_t nb[4];
  uint64_t stride[4];
  uint64_t nblocks;
};

// coefficient order by total sequency (sum of base-4 digits), stable in index:
// concatenation over s ascending of the indices whose digit sum is s
struct PermTable {
  int16_t p[4][256];
};
constexpr int digit_sum(int i, int d) {
  int s = 0;
  for (int a = 0; a < d; ++a) {
    s += i & 3;
    i >>= 2;
  }
  return s;
}
constexpr PermTable make_perm() {
  PermTable t{};
  for (int d = 1; d <= 4; ++d) {
    const int n = 1 << (2 * d);
    int k = 0;
    for (int s = 0; s <= 3 * d; ++s)
      for (int i = 0; i < n; ++i)
        if (digit_sum(i, d) == s) t.p[d - 1][k++] = (int16_t)i;
  }
  return t;
}
__constant__ PermTable kPerm = make_perm();

constexpr uint32_t NBMASK = 0xaaaaaaaau;

__device__ __forceinline__ uint32_t to_ordered(uint32_t b) {
  const uint32_t sign = 0x80000000u;
  return (b & sign) ? (b ^ (sign - 1)) : b;
}

__device__ __forceinline__ void fwd_lift(uint32_t* p, int s) {
  uint32_t x = p[0], y = p[s], z = p[2 * s], w = p[3 * s];
  w -= z; z -= y; y -= x;
  w -= z; z -= y;
  w -= z;
  p[0] = x; p[s] = y; p[2 * s] = z; p[3 * s] = w;
}
__device__ __forceinline__ void inv_lift(uint32_t* p, int s) {
  uint32_t x = p[0], y = p[s], z = p[2 * s], w = p[3 * s];
  w += z;
  z += y; w += z;
  y += x; z += y; w += z;
  p[0] = x; p[s] = y; p[2 * s] = z; p[3 * s] = w;
}

__device__ __forceinline__ void block_coords(const ZGeom& g, uint64_t b, uint32_t* bc) {
  for (int a = 0; a < 4; ++a) {
    bc[a] = (uint32_t)(b % g.nb[a]);
    b /= g.nb[a];
  }
}

struct BitOut {
  uint64_t* w;
  uint64_t cur = 0;
  int nbits = 0;
  uint32_t nw = 0;
  __device__ __forceinline__ void put(uint32_t bit) {
    cur |= (uint64_t)(bit & 1u) << nbits;
    if (++nbits == 64) {
      w[nw++] = cur;
      cur = 0;
      nbits = 0;
    }
  }
  __device__ __forceinline__ void flush() {
    if (nbits) {
      w[nw++] = cur;
      cur = 0;
      nbits = 0;
    }
  }
};

struct BitIn {
  const uint64_t* w;
  uint64_t cur;
  int left = 0;
  __device__ __forceinline__ uint32_t get() {
    if (left == 0) {
      cur = *w++;
      left = 64;
    }
    const uint32_t b = (uint32_t)(cur & 1ull);
    cur >>= 1;
    --left;
    return b;
  }
};

__global__ __launch_bounds__(64) void zfp_encode_kernel(const uint32_t* __restrict__ src, ZGeom g,
                                                        uint64_t* __restrict__ scratch, uint32_t maxw,
                                                        uint64_t* __restrict__ table) {
  const uint64_t b = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (b >= g.nblocks) return;
  const int n = 1 << (2 * g.d);
  uint32_t blk[256];
  uint32_t bc[4];
  block_coords(g, b, bc);
  for (int i = 0; i < n; ++i) {
    uint64_t off = 0;
    int c = i;
    for (int a = 0; a < g.d; ++a) {
      uint32_t x = bc[a] * 4 + (c & 3);
      c >>= 2;
      if (x >= g.shape[a]) x = g.shape[a] - 1;     // replicate the last sample
      off += x * g.stride[a];
    }
    blk[i] = to_ordered(src[off]);
  }
  for (int ax = 0; ax < g.d; ++ax) {
    const int s = 1 << (2 * ax);
    for (int base = 0; base < n; ++base)
      if (!((base >> (2 * ax)) & 3)) fwd_lift(blk + base, s);
  }
  uint32_t coef[256];
  for (int i = 0; i < n; ++i) coef[i] = (blk[kPerm.p[g.d - 1][i]] + NBMASK) ^ NBMASK;
  BitOut bo;
  bo.w = scratch + b * maxw;
  int nsig = 0;
  for (int k = 31; k >= 0; --k) {
    for (int i = 0; i < nsig; ++i) bo.put((coef[i] >> k) & 1u);
    while (nsig < n) {
      bool any = false;
      for (int i = nsig; i < n; ++i)
        if ((coef[i] >> k) & 1u) {
          any = true;
          break;
        }
      bo.put(any);
      if (!any) break;
      while (nsig < n - 1) {
        const uint32_t bit = (coef[nsig] >> k) & 1u;
        bo.put(bit);
        if (bit) break;
        ++nsig;
      }
      ++nsig;
    }
  }
  bo.flush();
  table[b] = bo.nw;
}

// exclusive scan of `n` u64 counts (one workgroup of 1024 threads); total -> *total
__global__ __launch_bounds__(1024) void zfp_scan_kernel(const uint64_t* __restrict__ cnt, uint64_t* __restrict__ offs,
                                                        uint64_t* __restrict__ total, uint64_t n) {
  __shared__ uint64_t part[1024];
  const int t = threadIdx.x;
  const uint64_t per = (n + 1023) / 1024;
  const uint64_t b0 = t * per, b1 = b0 + per < n ? b0 + per : n;
  uint64_t s = 0;
  for (uint64_t i = b0; i < b1; ++i) s += cnt[i];
  part[t] = s;
  __syncthreads();
  for (int d = 1; d < 1024; d <<= 1) {           // Hillis-Steele inclusive scan
    const uint64_t v = t >= d ? part[t - d] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  uint64_t run = t ? part[t - 1] : 0;
  for (uint64_t i = b0; i < b1; ++i) {
    offs[i] = run;
    run += cnt[i];
  }
  if (t == 1023) *total = part[1023];
}

__global__ __launch_bounds__(256) void zfp_pack_kernel(const uint64_t* __restrict__ scratch, uint32_t maxw,
                                                       const uint64_t* __restrict__ table,
                                                       const uint64_t* __restrict__ offs, uint64_t* __restrict__ out,
                                                       uint64_t nblocks) {
  const uint64_t b = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (b >= nblocks) return;
  const uint64_t nw = table[b];
  const uint64_t* s = scratch + b * maxw;
  uint64_t* o = out + offs[b];
  for (uint64_t i = 0; i < nw; ++i) o[i] = s[i];
}

__global__ __launch_bounds__(64) void zfp_decode_kernel(const uint64_t* __restrict__ words,
                                                        const uint64_t* __restrict__ offs, ZGeom g,
                                                        uint32_t* __restrict__ dst) {
  const uint64_t b = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (b >= g.nblocks) return;
  const int n = 1 << (2 * g.d);
  uint32_t coef[256];
  for (int i = 0; i < n; ++i) coef[i] = 0;
  BitIn bi;
  bi.w = words + offs[b];
  int nsig = 0;
  for (int k = 31; k >= 0; --k) {
    for (int i = 0; i < nsig; ++i) coef[i] |= bi.get() << k;
    while (nsig < n) {
      if (!bi.get()) break;
      while (nsig < n - 1) {
        if (bi.get()) break;
        ++nsig;
      }
      coef[nsig] |= 1u << k;
      ++nsig;
    }
  }
  uint32_t blk[256];
  for (int i = 0; i < n; ++i) blk[kPerm.p[g.d - 1][i]] = (coef[i] ^ NBMASK) - NBMASK;
  for (int ax = 0; ax < g.d; ++ax) {
    const int s = 1 << (2 * ax);
    for (int base = 0; base < n; ++base)
      if (!((base >> (2 * ax)) & 3)) inv_lift(blk + base, s);
  }
  uint32_t bc[4];
  block_coords(g, b, bc);
  for (int i = 0; i < n; ++i) {
    uint64_t off = 0;
    int c = i;
    bool ok = true;
    for (int a = 0; a < g.d; ++a) {
      const uint32_t x = bc[a] * 4 + (c & 3);
      c >>= 2;
      if (x >= g.shape[a]) {
        ok = false;
        break;
      }
      off += x * g.stride[a];
    }
    if (ok) dst[off] = to_ordered(blk[i]);         // the order map is an involution
  }
}

bool make_geom(const int64_t* shape_c, int nd, ZGeom* g) {
  if (nd < 1 || nd > 4) return false;
  g->d = nd;
  g->nblocks = 1;
  for (int a = 0; a < 4; ++a) {
    g->shape[a] = 1;
    g->nb[a] = 1;
  }
  for (int a = 0; a < nd; ++a) {
    const int64_t v = shape_c[nd - 1 - a];
    if (v <= 0 || v > 0xFFFFFFFFll) return false;
    g->shape[a] = (uint32_t)v;
    g->nb[a] = (uint32_t)((v + 3) / 4);
    g->nblocks *= g->nb[a];
  }
  g->stride[0] = 1;
  for (int a = 1; a < 4; ++a) g->stride[a] = g->stride[a - 1] * g->shape[a - 1];
  return true;
}

}  // namespace

uint32_t zfp_gpu_maxw(int nd) {
  const uint32_t n = 1u << (2 * nd);
  return (32 * n + 2 * n + 32 + 63) / 64;      // bit planes + scan bits + group tests (zfp_rev.cpp bound)
}

uint64_t zfp_gpu_nblocks(const int64_t* shape, int nd) {
  ZGeom g;
  return make_geom(shape, nd, &g) ? g.nblocks : 0;
}

// out = [nblocks x u64 word counts][payload words]; *total = payload words
hipError_t zfp_gpu_compress(const float* src, const int64_t* shape, int nd, uint64_t* scratch, uint64_t* offs,
                            uint64_t* out, uint64_t* total, hipStream_t s) {
  ZGeom g;
  if (!make_geom(shape, nd, &g)) return hipErrorInvalidValue;
  const uint32_t maxw = zfp_gpu_maxw(nd);
  const unsigned nb = (unsigned)((g.nblocks + 63) / 64);
  hipLaunchKernelGGL(zfp_encode_kernel, dim3(nb), dim3(64), 0, s, (const uint32_t*)src, g, scratch, maxw, out);
  hipLaunchKernelGGL(zfp_scan_kernel, dim3(1), dim3(1024), 0, s, out, offs, total, g.nblocks);
  hipLaunchKernelGGL(zfp_pack_kernel, dim3((unsigned)((g.nblocks + 255) / 256)), dim3(256), 0, s, scratch, maxw,
                     out, offs, out + g.nblocks, g.nblocks);
  return hipGetLastError();
}

// table = nblocks u64 word counts followed by the payload words (a host container minus its header)
hipError_t zfp_gpu_decompress(const uint64_t* table, const int64_t* shape, int nd, uint64_t* offs, uint64_t* total,
                              float* dst, hipStream_t s) {
  ZGeom g;
  if (!make_geom(shape, nd, &g)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(zfp_scan_kernel, dim3(1), dim3(1024), 0, s, table, offs, total, g.nblocks);
  hipLaunchKernelGGL(zfp_decode_kernel, dim3((unsigned)((g.nblocks + 63) / 64)), dim3(64), 0, s,
                     table + g.nblocks, offs, g, (uint32_t*)dst);
  return hipGetLastError();
}

}  // namespace adapt
