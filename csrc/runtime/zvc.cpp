// Host encoder/decoder for the "AZVC" zero-value-compression stream produced by
// csrc/kernels/zvc_gpu.hip (same byte format), so CPU stages and the
// dispatcher can read GPU-compressed activations and vice versa.
#include <cstring>
#include <stdexcept>

#include "runtime.h"

namespace adapt_rt {

static const int ZSEG = 4096, ZGROUPS = ZSEG / 64, ZHDR = 32;

std::vector<uint8_t> zvc_compress(const uint8_t* in, size_t n, int esz) {
  if (esz != 2 && esz != 4) throw std::runtime_error("zvc: element size must be 2 or 4");
  const size_t nseg = (n + ZSEG - 1) / ZSEG;
  std::vector<uint8_t> out(ZHDR + 4 * nseg);
  out.reserve(ZHDR + 4 * nseg + nseg * ZGROUPS * 8 + n * esz);
  std::memcpy(out.data(), "AZVC", 4);
  out[4] = 1;
  out[5] = (uint8_t)esz;
  uint64_t nn = n;
  std::memcpy(out.data() + 8, &nn, 8);
  uint32_t seg = ZSEG, ns = (uint32_t)nseg;
  std::memcpy(out.data() + 16, &seg, 4);
  std::memcpy(out.data() + 20, &ns, 4);
  for (size_t s = 0; s < nseg; ++s) {
    const size_t start = out.size();
    std::vector<uint8_t> vals;
    for (int g = 0; g < ZGROUPS; ++g) {
      uint64_t mask = 0;
      for (int l = 0; l < 64; ++l) {
        const size_t i = s * ZSEG + (size_t)g * 64 + l;
        if (i >= n) break;
        const uint8_t* p = in + i * esz;
        bool nz = false;
        for (int b = 0; b < esz; ++b) nz |= p[b] != 0;
        if (nz) {
          mask |= 1ull << l;
          vals.insert(vals.end(), p, p + esz);
        }
      }
      const uint8_t* mb = reinterpret_cast<const uint8_t*>(&mask);
      out.insert(out.end(), mb, mb + 8);
    }
    out.insert(out.end(), vals.begin(), vals.end());
    const uint32_t sz = (uint32_t)(out.size() - start);
    std::memcpy(out.data() + ZHDR + 4 * s, &sz, 4);
  }
  return out;
}

ZvcHeader zvc_header(const uint8_t* p, size_t len) {
  if (len < (size_t)ZHDR || std::memcmp(p, "AZVC", 4) != 0) throw std::runtime_error("zvc: bad magic");
  ZvcHeader h;
  h.esz = p[5];
  std::memcpy(&h.n, p + 8, 8);
  uint32_t seg, ns;
  std::memcpy(&seg, p + 16, 4);
  std::memcpy(&ns, p + 20, 4);
  if (seg != (uint32_t)ZSEG || (h.esz != 2 && h.esz != 4) || ns != (h.n + ZSEG - 1) / ZSEG)
    throw std::runtime_error("zvc: bad header");
  if (len < (size_t)ZHDR + 4ull * ns) throw std::runtime_error("zvc: truncated size table");
  h.nseg = ns;
  uint32_t acc = 0;
  for (uint32_t s = 0; s < ns; ++s) {
    uint32_t sz;
    std::memcpy(&sz, p + ZHDR + 4 * s, 4);
    h.offsets.push_back(acc);
    acc += sz;
  }
  if (len < (size_t)ZHDR + 4ull * ns + acc) throw std::runtime_error("zvc: truncated payload");
  return h;
}

void zvc_decompress(const uint8_t* p, size_t len, uint8_t* out) {
  ZvcHeader h = zvc_header(p, len);
  const uint8_t* body = p + ZHDR + 4ull * h.nseg;
  const int esz = h.esz;
  for (uint32_t s = 0; s < h.nseg; ++s) {
    const uint8_t* seg = body + h.offsets[s];
    const uint8_t* vals = seg + ZGROUPS * 8;
    for (int g = 0; g < ZGROUPS; ++g) {
      uint64_t mask;
      std::memcpy(&mask, seg + g * 8, 8);
      for (int l = 0; l < 64; ++l) {
        const size_t i = (size_t)s * ZSEG + (size_t)g * 64 + l;
        if (i >= h.n) break;
        if ((mask >> l) & 1ull) {
          std::memcpy(out + i * esz, vals, esz);
          vals += esz;
        } else {
          std::memset(out + i * esz, 0, esz);
        }
      }
    }
  }
}

}  // namespace adapt_rt
