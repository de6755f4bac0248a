// LZ4 block + frame codec (host, C++17), written from the public format
// specifications (LZ4 Block Format 1.6.x, LZ4 Frame Format 1.6.x, xxHash32).
//
// The reference compresses every weight array and activation with
// `lz4.frame.compress(zfpy.compress_numpy(arr))` (`src/dispatcher.py:92-98`,
// `src/node.py:122-125`).  This is our native replacement: a greedy
// hash-chain-free LZ4 compressor (single 4-byte hash table, like lz4 "fast"),
// a bounds-checked decompressor, and the frame container (magic 0x184D2204,
// independent 4 MiB blocks, content size + content checksum) so frames are
// readable by any standard LZ4 frame decoder.
#include "runtime.h"

#include <cstring>
#include <stdexcept>
#include <vector>

namespace adapt_rt {

// ------------------------------------------------------------- xxHash32
static inline uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
static const uint32_t P1 = 2654435761U, P2 = 2246822519U, P3 = 3266489917U, P4 = 668265263U, P5 = 374761393U;
static inline uint32_t rd32(const uint8_t* p) { uint32_t v; std::memcpy(&v, p, 4); return v; }
static inline uint16_t rd16(const uint8_t* p) { uint16_t v; std::memcpy(&v, p, 2); return v; }
static inline void wr32(uint8_t* p, uint32_t v) { std::memcpy(p, &v, 4); }
static inline void wr16(uint8_t* p, uint16_t v) { std::memcpy(p, &v, 2); }

uint32_t xxh32(const uint8_t* p, size_t len, uint32_t seed) {
  const uint8_t* end = p + len;
  uint32_t h;
  if (len >= 16) {
    uint32_t v1 = seed + P1 + P2, v2 = seed + P2, v3 = seed, v4 = seed - P1;
    const uint8_t* lim = end - 16;
    do {
      v1 = rotl32(v1 + rd32(p) * P2, 13) * P1; p += 4;
      v2 = rotl32(v2 + rd32(p) * P2, 13) * P1; p += 4;
      v3 = rotl32(v3 + rd32(p) * P2, 13) * P1; p += 4;
      v4 = rotl32(v4 + rd32(p) * P2, 13) * P1; p += 4;
    } while (p <= lim);
    h = rotl32(v1, 1) + rotl32(v2, 7) + rotl32(v3, 12) + rotl32(v4, 18);
  } else {
    h = seed + P5;
  }
  h += (uint32_t)len;
  while (p + 4 <= end) { h = rotl32(h + rd32(p) * P3, 17) * P4; p += 4; }
  while (p < end) { h = rotl32(h + (*p) * P5, 11) * P1; ++p; }
  h ^= h >> 15; h *= P2; h ^= h >> 13; h *= P3; h ^= h >> 16;
  return h;
}

// ------------------------------------------------------------ LZ4 block
static const int MINMATCH = 4;
static const int LASTLITERALS = 5;     // last 5 bytes are always literals
static const int MFLIMIT = 12;         // no match may start within the last 12 bytes
static const int HASH_LOG = 16;

static inline uint32_t hash4(uint32_t v) { return (v * 2654435761U) >> (32 - HASH_LOG); }

size_t lz4_block_bound(size_t n) { return n + n / 255 + 16; }

static inline uint8_t* put_len(uint8_t* op, size_t len) {
  while (len >= 255) { *op++ = 255; len -= 255; }
  *op++ = (uint8_t)len;
  return op;
}

size_t lz4_block_compress(const uint8_t* src, size_t n, uint8_t* dst, size_t cap, int accel) {
  if (cap < lz4_block_bound(n)) throw std::runtime_error("lz4: output capacity too small");
  uint8_t* op = dst;
  const uint8_t* ip = src;
  const uint8_t* anchor = src;
  const uint8_t* iend = src + n;
  if (n < (size_t)MFLIMIT + 1) goto last_literals;
  {
    std::vector<uint32_t> table(1u << HASH_LOG, 0);
    const uint8_t* mflimit = iend - MFLIMIT;
    const uint8_t* matchlimit = iend - LASTLITERALS;
    if (accel < 1) accel = 1;
    ip++;
    while (ip < mflimit) {
      // find a match (skip faster over incompressible data)
      const uint8_t* match = nullptr;
      int step = 1, search = accel << 6;
      for (;;) {
        uint32_t h = hash4(rd32(ip));
        match = src + table[h];
        table[h] = (uint32_t)(ip - src);
        if (match < ip && ip - match <= 65535 && rd32(match) == rd32(ip)) break;
        ip += step;
        step = (search++ >> 6);
        if (ip >= mflimit) goto last_literals;
      }
      // extend backwards
      while (ip > anchor && match > src && ip[-1] == match[-1]) { ip--; match--; }
      // extend forwards
      const uint8_t* p = ip + MINMATCH;
      const uint8_t* m = match + MINMATCH;
      while (p < matchlimit && *p == *m) { p++; m++; }
      size_t lit = (size_t)(ip - anchor);
      size_t mlen = (size_t)(p - ip) - MINMATCH;
      uint8_t* token = op++;
      *token = (uint8_t)((lit >= 15 ? 15 : lit) << 4);
      if (lit >= 15) op = put_len(op, lit - 15);
      std::memcpy(op, anchor, lit);
      op += lit;
      wr16(op, (uint16_t)(ip - match));
      op += 2;
      *token |= (uint8_t)(mlen >= 15 ? 15 : mlen);
      if (mlen >= 15) op = put_len(op, mlen - 15);
      // index a position inside the match to help the next search
      if (p - 2 > src) table[hash4(rd32(p - 2))] = (uint32_t)(p - 2 - src);
      ip = p;
      anchor = ip;
    }
  }
last_literals: {
  size_t lit = (size_t)(iend - anchor);
  uint8_t* token = op++;
  *token = (uint8_t)((lit >= 15 ? 15 : lit) << 4);
  if (lit >= 15) op = put_len(op, lit - 15);
  std::memcpy(op, anchor, lit);
  op += lit;
}
  return (size_t)(op - dst);
}

size_t lz4_block_decompress(const uint8_t* src, size_t n, uint8_t* dst, size_t cap) {
  const uint8_t* ip = src;
  const uint8_t* iend = src + n;
  uint8_t* op = dst;
  uint8_t* oend = dst + cap;
  while (ip < iend) {
    unsigned token = *ip++;
    size_t lit = token >> 4;
    if (lit == 15) {
      unsigned b;
      do {
        if (ip >= iend) throw std::runtime_error("lz4: truncated literal length");
        b = *ip++;
        lit += b;
      } while (b == 255);
    }
    if ((size_t)(iend - ip) < lit || (size_t)(oend - op) < lit) throw std::runtime_error("lz4: literal overrun");
    std::memcpy(op, ip, lit);
    op += lit;
    ip += lit;
    if (ip >= iend) break;       // last sequence has no match
    if (iend - ip < 2) throw std::runtime_error("lz4: truncated offset");
    size_t off = rd16(ip);
    ip += 2;
    if (off == 0 || off > (size_t)(op - dst)) throw std::runtime_error("lz4: bad match offset");
    size_t mlen = token & 15;
    if (mlen == 15) {
      unsigned b;
      do {
        if (ip >= iend) throw std::runtime_error("lz4: truncated match length");
        b = *ip++;
        mlen += b;
      } while (b == 255);
    }
    mlen += MINMATCH;
    if ((size_t)(oend - op) < mlen) throw std::runtime_error("lz4: match overrun");
    const uint8_t* m = op - off;
    if (off >= mlen) {
      std::memcpy(op, m, mlen);
      op += mlen;
    } else {
      for (size_t i = 0; i < mlen; ++i) op[i] = m[i];   // overlapping copy
      op += mlen;
    }
  }
  return (size_t)(op - dst);
}

// ------------------------------------------------------------ LZ4 frame
static const uint32_t LZ4F_MAGIC = 0x184D2204U;
static const size_t FRAME_BLOCK = 4u << 20;   // BD = 7 (4 MiB max block)

std::vector<uint8_t> lz4_frame_compress(const uint8_t* src, size_t n, int accel) {
  std::vector<uint8_t> out;
  out.reserve(15 + n + n / 255 + 64);
  uint8_t hdr[15];
  wr32(hdr, LZ4F_MAGIC);
  // FLG: version 01, block independence 1, block checksum 0, content size 1, content checksum 1
  uint8_t flg = (1u << 6) | (1u << 5) | (1u << 3) | (1u << 2);
  uint8_t bd = 7u << 4;
  hdr[4] = flg;
  hdr[5] = bd;
  uint64_t cs = n;
  std::memcpy(hdr + 6, &cs, 8);
  hdr[14] = (uint8_t)((xxh32(hdr + 4, 10, 0) >> 8) & 0xFF);
  out.insert(out.end(), hdr, hdr + 15);
  std::vector<uint8_t> tmp(lz4_block_bound(FRAME_BLOCK));
  for (size_t off = 0; off < n; off += FRAME_BLOCK) {
    size_t len = std::min(FRAME_BLOCK, n - off);
    size_t c = lz4_block_compress(src + off, len, tmp.data(), tmp.size(), accel);
    uint8_t bs[4];
    if (c >= len) {   // store uncompressed
      wr32(bs, (uint32_t)len | 0x80000000U);
      out.insert(out.end(), bs, bs + 4);
      out.insert(out.end(), src + off, src + off + len);
    } else {
      wr32(bs, (uint32_t)c);
      out.insert(out.end(), bs, bs + 4);
      out.insert(out.end(), tmp.data(), tmp.data() + c);
    }
  }
  uint8_t endmark[4] = {0, 0, 0, 0};
  out.insert(out.end(), endmark, endmark + 4);
  uint8_t ck[4];
  wr32(ck, xxh32(src, n, 0));
  out.insert(out.end(), ck, ck + 4);
  return out;
}

Lz4FrameBlocks lz4_frame_blocks(const uint8_t* src, size_t n) {
  Lz4FrameBlocks r;
  if (n < 7 || rd32(src) != LZ4F_MAGIC) throw std::runtime_error("lz4f: bad magic");
  uint8_t flg = src[4], bd = src[5];
  bool bchk = flg & (1u << 4), has_cs = flg & (1u << 3), dict = flg & 1u;
  size_t hlen = 2 + (has_cs ? 8 : 0) + (dict ? 4 : 0);
  if (n < 4 + hlen + 1) throw std::runtime_error("lz4f: truncated header");
  r.independent = flg & (1u << 5);
  r.block_max = (size_t)1 << (8 + 2 * ((bd >> 4) & 7));
  r.content_size = 0;
  if (has_cs) std::memcpy(&r.content_size, src + 6, 8);
  size_t pos = 4 + hlen + 1;
  for (;;) {
    if (n - pos < 4) throw std::runtime_error("lz4f: truncated block size");
    uint32_t bs = rd32(src + pos);
    pos += 4;
    if (bs == 0) break;
    size_t len = bs & 0x7FFFFFFFU;
    if (n - pos < len) throw std::runtime_error("lz4f: truncated block");
    r.offsets.push_back((uint32_t)pos);
    r.words.push_back(bs);
    pos += len + (bchk ? 4 : 0);
  }
  return r;
}

std::vector<uint8_t> lz4_frame_decompress(const uint8_t* src, size_t n) {
  std::vector<uint8_t> out;
  size_t pos = 0;
  while (pos < n) {    // concatenated frames are allowed
    if (n - pos < 7) throw std::runtime_error("lz4f: truncated header");
    uint32_t magic = rd32(src + pos);
    if ((magic & 0xFFFFFFF0U) == 0x184D2A50U) {   // skippable frame
      if (n - pos < 8) throw std::runtime_error("lz4f: truncated skippable frame");
      uint32_t sz = rd32(src + pos + 4);
      pos += 8 + (size_t)sz;
      continue;
    }
    if (magic != LZ4F_MAGIC) throw std::runtime_error("lz4f: bad magic");
    uint8_t flg = src[pos + 4], bd = src[pos + 5];
    if ((flg >> 6) != 1) throw std::runtime_error("lz4f: unsupported version");
    bool bchk = flg & (1u << 4), has_cs = flg & (1u << 3), cchk = flg & (1u << 2), dict = flg & 1u;
    size_t hlen = 2 + (has_cs ? 8 : 0) + (dict ? 4 : 0);
    if (n - pos < 4 + hlen + 1) throw std::runtime_error("lz4f: truncated header");
    uint8_t hc = (uint8_t)((xxh32(src + pos + 4, hlen, 0) >> 8) & 0xFF);
    if (hc != src[pos + 4 + hlen]) throw std::runtime_error("lz4f: header checksum mismatch");
    int bid = (bd >> 4) & 7;
    if (bid < 4) throw std::runtime_error("lz4f: bad block size id");
    size_t bmax = (size_t)1 << (8 + 2 * bid);
    uint64_t content = 0;
    if (has_cs) std::memcpy(&content, src + pos + 6, 8);
    pos += 4 + hlen + 1;
    size_t start = out.size();
    if (has_cs) out.reserve(start + content);
    bool linked = !(flg & (1u << 5));
    for (;;) {
      if (n - pos < 4) throw std::runtime_error("lz4f: truncated block size");
      uint32_t bs = rd32(src + pos);
      pos += 4;
      if (bs == 0) break;
      bool raw = bs & 0x80000000U;
      size_t len = bs & 0x7FFFFFFFU;
      if (n - pos < len + (bchk ? 4 : 0)) throw std::runtime_error("lz4f: truncated block");
      if (raw) {
        out.insert(out.end(), src + pos, src + pos + len);
      } else {
        size_t o = out.size();
        if (linked) {
          // linked blocks may reference up to 64 KiB of previous output: decode in place
          out.resize(o + bmax);
          size_t prefix = std::min<size_t>(o - start, 65536);
          // decode with the previous output as dictionary: copy window ahead of the buffer
          std::vector<uint8_t> win(prefix + bmax);
          std::memcpy(win.data(), out.data() + o - prefix, prefix);
          // run the decoder on win starting after the prefix (offset check is relative to win start)
          const uint8_t* ip = src + pos;
          size_t got = 0;
          {
            // inline decoder allowing references into the prefix
            const uint8_t* iend = ip + len;
            uint8_t* op = win.data() + prefix;
            uint8_t* oend = win.data() + win.size();
            while (ip < iend) {
              unsigned token = *ip++;
              size_t lit = token >> 4;
              if (lit == 15) { unsigned b; do { b = *ip++; lit += b; } while (b == 255 && ip < iend); }
              if ((size_t)(iend - ip) < lit || (size_t)(oend - op) < lit) throw std::runtime_error("lz4f: literal overrun");
              std::memcpy(op, ip, lit); op += lit; ip += lit;
              if (ip >= iend) break;
              size_t off = rd16(ip); ip += 2;
              if (off == 0 || off > (size_t)(op - win.data())) throw std::runtime_error("lz4f: bad offset");
              size_t mlen = token & 15;
              if (mlen == 15) { unsigned b; do { b = *ip++; mlen += b; } while (b == 255 && ip < iend); }
              mlen += MINMATCH;
              if ((size_t)(oend - op) < mlen) throw std::runtime_error("lz4f: match overrun");
              uint8_t* m = op - off;
              for (size_t i = 0; i < mlen; ++i) op[i] = m[i];
              op += mlen;
            }
            got = (size_t)(op - (win.data() + prefix));
          }
          std::memcpy(out.data() + o, win.data() + prefix, got);
          out.resize(o + got);
        } else {
          out.resize(o + bmax);
          size_t got = lz4_block_decompress(src + pos, len, out.data() + o, bmax);
          out.resize(o + got);
        }
      }
      pos += len;
      if (bchk) {
        uint32_t want = rd32(src + pos);
        const uint8_t* blk = src + pos - len;
        if (xxh32(blk, len, 0) != want) throw std::runtime_error("lz4f: block checksum mismatch");
        pos += 4;
      }
    }
    if (cchk) {
      if (n - pos < 4) throw std::runtime_error("lz4f: truncated content checksum");
      uint32_t want = rd32(src + pos);
      pos += 4;
      if (xxh32(out.data() + start, out.size() - start, 0) != want)
        throw std::runtime_error("lz4f: content checksum mismatch");
    }
    if (has_cs && out.size() - start != content) throw std::runtime_error("lz4f: content size mismatch");
  }
  return out;
}

}  // namespace adapt_rt
