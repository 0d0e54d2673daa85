// LZ4 frame codec (host code) for the reth_buffer wire format's compressed messages.
//
// Client.append(..., compress=True) -- what test/apex-dqn/worker.py:60 sends -- wraps the
// message body in an LZ4 frame (reth_buffer/reth_buffer/utils/pack.py:62-84, python-lz4's
// lz4.frame.compress: version 01, block max size from BD, independent or linked blocks,
// optional content size, content checksum and block checksums).  No lz4 library is in this
// image, so the published format is restated here: frame = magic 0x184D2204, FLG, BD,
// [content size u64], [dict id u32], header checksum = (xxh32(descriptor) >> 8) & 0xff;
// blocks = u32 size (bit 31 = stored uncompressed) + data [+ xxh32 block checksum];
// end mark 0; [xxh32 content checksum].  A block is a run of sequences: token (literal
// length hi nibble, match length - 4 lo nibble, 15 = continued in 255-bytes), literals,
// u16 little-endian offset, match copy (may overlap its own output).  The encoder is a
// greedy single-hash matcher producing standard frames (independent 4 MB blocks, content
// size and content checksum stored); any LZ4 decoder reads them.
#include <cstdint>
#include <cstring>
#include <vector>

#include "common.hpp"

namespace {

constexpr uint32_t kMagic = 0x184D2204u;
constexpr uint32_t P1 = 2654435761u, P2 = 2246822519u, P3 = 3266489917u, P4 = 668265263u, P5 = 374761393u;

inline uint32_t rotl(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
inline uint32_t rd32(const uint8_t *p) { uint32_t v; std::memcpy(&v, p, 4); return v; }  // little-endian host
inline void wr32(uint8_t *p, uint32_t v) { std::memcpy(p, &v, 4); }

uint32_t xxh32(const uint8_t *p, size_t len, uint32_t seed) {
  const uint8_t *end = p + len;
  uint32_t h;
  if (len >= 16) {
    uint32_t v1 = seed + P1 + P2, v2 = seed + P2, v3 = seed, v4 = seed - P1;
    const uint8_t *limit = end - 16;
    do {
      v1 = rotl(v1 + rd32(p) * P2, 13) * P1;
      v2 = rotl(v2 + rd32(p + 4) * P2, 13) * P1;
      v3 = rotl(v3 + rd32(p + 8) * P2, 13) * P1;
      v4 = rotl(v4 + rd32(p + 12) * P2, 13) * P1;
      p += 16;
    } while (p <= limit);
    h = rotl(v1, 1) + rotl(v2, 7) + rotl(v3, 12) + rotl(v4, 18);
  } else {
    h = seed + P5;
  }
  h += (uint32_t)len;
  while (p + 4 <= end) {
    h = rotl(h + rd32(p) * P3, 17) * P4;
    p += 4;
  }
  while (p < end) {
    h = rotl(h + (*p) * P5, 11) * P1;
    ++p;
  }
  h ^= h >> 15;
  h *= P2;
  h ^= h >> 13;
  h *= P3;
  h ^= h >> 16;
  return h;
}

struct FrameInfo {
  bool block_checksum, content_checksum, has_size;
  int64_t content_size, block_max;
  size_t header_len;
};

int parse_header(const uint8_t *src, int64_t n, FrameInfo *fi) {
  RTH_REQUIRE(n >= 7 && rd32(src) == kMagic, "lz4 frame: bad magic");
  const uint8_t flg = src[4], bd = src[5];
  RTH_REQUIRE((flg >> 6) == 1, "lz4 frame: unsupported version %d", flg >> 6);
  fi->block_checksum = flg & 0x10;
  fi->has_size = flg & 0x08;
  fi->content_checksum = flg & 0x04;
  const bool dict = flg & 0x01;
  const int bsid = (bd >> 4) & 7;
  RTH_REQUIRE(bsid >= 4, "lz4 frame: bad block max size id %d", bsid);
  fi->block_max = int64_t(1) << (8 + 2 * bsid);  // 4: 64 KB ... 7: 4 MB
  size_t pos = 6;
  fi->content_size = -1;
  if (fi->has_size) {
    RTH_REQUIRE(n >= (int64_t)(pos + 8 + 1), "lz4 frame: truncated header");
    uint64_t s;
    std::memcpy(&s, src + pos, 8);
    fi->content_size = (int64_t)s;
    pos += 8;
  }
  if (dict) pos += 4;
  RTH_REQUIRE(n >= (int64_t)(pos + 1), "lz4 frame: truncated header");
  const uint8_t hc = (uint8_t)((xxh32(src + 4, pos - 4, 0) >> 8) & 0xff);
  RTH_REQUIRE(hc == src[pos], "lz4 frame: header checksum mismatch");
  fi->header_len = pos + 1;
  return RTH_OK;
}

// one compressed block into dst[*o .. cap), matches may reach back into earlier output
int decode_block(const uint8_t *s, size_t len, uint8_t *dst, int64_t cap, int64_t *o) {
  size_t i = 0;
  int64_t out = *o;
  while (i < len) {
    const uint8_t tok = s[i++];
    size_t lit = tok >> 4;
    if (lit == 15) {
      uint8_t b;
      do {
        RTH_REQUIRE(i < len, "lz4 block: truncated literal length");
        b = s[i++];
        lit += b;
      } while (b == 255);
    }
    RTH_REQUIRE(i + lit <= len && out + (int64_t)lit <= cap, "lz4 block: literals overrun");
    std::memcpy(dst + out, s + i, lit);
    i += lit;
    out += lit;
    if (i == len) break;  // the last sequence has literals only
    RTH_REQUIRE(i + 2 <= len, "lz4 block: truncated offset");
    const size_t off = s[i] | (s[i + 1] << 8);
    i += 2;
    RTH_REQUIRE(off >= 1 && (int64_t)off <= out, "lz4 block: offset %zu outside the output", off);
    size_t ml = (tok & 15) + 4;
    if ((tok & 15) == 15) {
      uint8_t b;
      do {
        RTH_REQUIRE(i < len, "lz4 block: truncated match length");
        b = s[i++];
        ml += b;
      } while (b == 255);
    }
    RTH_REQUIRE(out + (int64_t)ml <= cap, "lz4 block: match overruns the output");
    const uint8_t *from = dst + out - off;
    for (size_t k = 0; k < ml; ++k) dst[out + k] = from[k];  // byte order: overlapping copies repeat
    out += ml;
  }
  *o = out;
  return RTH_OK;
}

void put_len(std::vector<uint8_t> &v, size_t x) {  // the 255-continuation of a length past 15
  while (x >= 255) {
    v.push_back(255);
    x -= 255;
  }
  v.push_back((uint8_t)x);
}

void encode_block(const uint8_t *src, size_t n, std::vector<uint8_t> &out) {
  constexpr int kHashLog = 16;
  std::vector<int32_t> table(size_t(1) << kHashLog, -1);
  auto hash = [](uint32_t v) { return (v * 2654435761u) >> (32 - kHashLog); };
  size_t anchor = 0, i = 0;
  // the format: the last match starts >= 12 bytes before the end, the last 5 bytes are literals
  const size_t match_limit = n > 12 ? n - 12 : 0;
  auto emit = [&](size_t lit_end, size_t off, size_t mlen) {
    const size_t lit = lit_end - anchor;
    const size_t ml = mlen ? mlen - 4 : 0;
    out.push_back((uint8_t)(((lit < 15 ? lit : 15) << 4) | (mlen ? (ml < 15 ? ml : 15) : 0)));
    if (lit >= 15) put_len(out, lit - 15);
    out.insert(out.end(), src + anchor, src + lit_end);
    if (mlen) {
      out.push_back((uint8_t)(off & 0xff));
      out.push_back((uint8_t)(off >> 8));
      if (ml >= 15) put_len(out, ml - 15);
    }
  };
  while (i < match_limit) {
    const uint32_t v = rd32(src + i);
    const uint32_t hk = hash(v);
    const int32_t cand = table[hk];
    table[hk] = (int32_t)i;
    if (cand >= 0 && i - (size_t)cand <= 65535 && rd32(src + cand) == v) {
      size_t m = 4;
      const size_t max_m = n - 5 - i;  // leave the last 5 bytes as literals
      while (m < max_m && src[cand + m] == src[i + m]) ++m;
      emit(i, i - (size_t)cand, m);
      i += m;
      anchor = i;
    } else {
      ++i;
    }
  }
  emit(n, 0, 0);
}

}  // namespace

extern "C" {

// the decompressed size of a frame: its stored content size, or an upper bound (blocks x
// block max size) when the frame does not store it
int rth_lz4_frame_bound(const uint8_t *src, int64_t n, int64_t *bound) {
  RTH_REQUIRE(src && bound, "rth_lz4_frame_bound: NULL argument");
  FrameInfo fi;
  int rc = parse_header(src, n, &fi);
  if (rc) return rc;
  if (fi.has_size) {
    *bound = fi.content_size;
    return RTH_OK;
  }
  int64_t total = 0;
  size_t pos = fi.header_len;
  for (;;) {
    RTH_REQUIRE((int64_t)pos + 4 <= n, "lz4 frame: truncated block size");
    const uint32_t bs = rd32(src + pos);
    pos += 4;
    if (bs == 0) break;
    const size_t len = bs & 0x7fffffffu;
    pos += len + (fi.block_checksum ? 4 : 0);
    RTH_REQUIRE((int64_t)pos <= n, "lz4 frame: truncated block");
    total += fi.block_max;
  }
  *bound = total;
  return RTH_OK;
}

int rth_lz4_frame_decompress(const uint8_t *src, int64_t n, uint8_t *dst, int64_t cap, int64_t *out_len) {
  RTH_REQUIRE(src && out_len && (dst || cap == 0), "rth_lz4_frame_decompress: NULL argument");
  FrameInfo fi;
  int rc = parse_header(src, n, &fi);
  if (rc) return rc;
  size_t pos = fi.header_len;
  int64_t out = 0;
  for (;;) {
    RTH_REQUIRE((int64_t)pos + 4 <= n, "lz4 frame: truncated block size");
    const uint32_t bs = rd32(src + pos);
    pos += 4;
    if (bs == 0) break;  // end mark
    const size_t len = bs & 0x7fffffffu;
    RTH_REQUIRE((int64_t)(pos + len + (fi.block_checksum ? 4 : 0)) <= n, "lz4 frame: truncated block");
    if (fi.block_checksum)
      RTH_REQUIRE(xxh32(src + pos, len, 0) == rd32(src + pos + len), "lz4 frame: block checksum mismatch");
    const int64_t before = out;
    if (bs & 0x80000000u) {  // stored
      RTH_REQUIRE(out + (int64_t)len <= cap, "lz4 frame: output buffer too small");
      std::memcpy(dst + out, src + pos, len);
      out += len;
    } else {
      rc = decode_block(src + pos, len, dst, cap, &out);
      if (rc) return rc;
    }
    RTH_REQUIRE(out - before <= fi.block_max, "lz4 frame: block larger than the block max size");
    pos += len + (fi.block_checksum ? 4 : 0);
  }
  if (fi.content_checksum) {
    RTH_REQUIRE((int64_t)pos + 4 <= n, "lz4 frame: truncated content checksum");
    RTH_REQUIRE(xxh32(dst, (size_t)out, 0) == rd32(src + pos), "lz4 frame: content checksum mismatch");
    pos += 4;
  }
  RTH_REQUIRE(!fi.has_size || fi.content_size == out, "lz4 frame: content size %lld, decoded %lld",
              (long long)fi.content_size, (long long)out);
  *out_len = out;
  return RTH_OK;
}

// worst-case encoded size of n bytes (the caller's output capacity)
int64_t rth_lz4_frame_compress_bound(int64_t n) {
  const int64_t blocks = n / (int64_t(4) << 20) + 1;
  return 19 + n + n / 255 + blocks * 24 + 16;
}

int rth_lz4_frame_compress(const uint8_t *src, int64_t n, uint8_t *dst, int64_t cap, int64_t *out_len) {
  RTH_REQUIRE((src || n == 0) && dst && out_len && n >= 0, "rth_lz4_frame_compress: bad arguments");
  std::vector<uint8_t> f;
  f.reserve((size_t)n / 2 + 64);
  f.resize(4);
  wr32(f.data(), kMagic);
  f.push_back(0x40 | 0x20 | 0x08 | 0x04);  // version 01, independent blocks, content size, content checksum
  f.push_back(7 << 4);                       // 4 MB blocks
  const uint64_t cs = (uint64_t)n;
  for (int k = 0; k < 8; ++k) f.push_back((uint8_t)(cs >> (8 * k)));
  f.push_back((uint8_t)((xxh32(f.data() + 4, f.size() - 4, 0) >> 8) & 0xff));
  const int64_t bmax = int64_t(4) << 20;
  std::vector<uint8_t> blk;
  for (int64_t at = 0; at < n; at += bmax) {
    const size_t len = (size_t)(n - at < bmax ? n - at : bmax);
    blk.clear();
    encode_block(src + at, len, blk);
    uint8_t sz[4];
    if (blk.size() >= len) {  // incompressible: stored
      wr32(sz, (uint32_t)len | 0x80000000u);
      f.insert(f.end(), sz, sz + 4);
      f.insert(f.end(), src + at, src + at + len);
    } else {
      wr32(sz, (uint32_t)blk.size());
      f.insert(f.end(), sz, sz + 4);
      f.insert(f.end(), blk.begin(), blk.end());
    }
  }
  uint8_t tail[8];
  wr32(tail, 0);
  wr32(tail + 4, xxh32(src, (size_t)n, 0));
  f.insert(f.end(), tail, tail + 8);
  RTH_REQUIRE((int64_t)f.size() <= cap, "rth_lz4_frame_compress: output buffer too small (%zu > %lld)", f.size(),
              (long long)cap);
  std::memcpy(dst, f.data(), f.size());
  *out_len = (int64_t)f.size();
  return RTH_OK;
}

uint32_t rth_xxh32(const uint8_t *src, int64_t n, uint32_t seed) { return xxh32(src, (size_t)n, seed); }

}  // extern "C"
