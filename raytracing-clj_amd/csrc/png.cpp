// png.cpp — PNG output for the host side: rt_write_png (8-bit RGB from the
// quantised frame) and rt_ppm_to_png, the behaviour of the reference's
// src/ppm2png.clj:35-87 (P3 in, 8-bit RGB PNG out).  Written from the PNG
// specification (signature, IHDR / IDAT / IEND chunks with CRC-32, zlib
// stream of per-row filtered scanlines); deflate and CRC come from zlib.
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <cctype>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "rt_internal.h"

namespace {

void put_u32(std::vector<uint8_t>& v, uint32_t x) {
  v.push_back(static_cast<uint8_t>(x >> 24));
  v.push_back(static_cast<uint8_t>(x >> 16));
  v.push_back(static_cast<uint8_t>(x >> 8));
  v.push_back(static_cast<uint8_t>(x));
}

// one chunk: length, type, data, CRC-32 over type + data
void chunk(std::vector<uint8_t>& out, const char type[4], const uint8_t* data, size_t n) {
  put_u32(out, static_cast<uint32_t>(n));
  const size_t at = out.size();
  out.insert(out.end(), type, type + 4);
  if (n) out.insert(out.end(), data, data + n);
  uLong crc = crc32(0L, Z_NULL, 0);
  crc = crc32(crc, out.data() + at, static_cast<uInt>(n + 4));
  put_u32(out, static_cast<uint32_t>(crc));
}

// scanlines with a filter byte each; per row the filter (None, Sub, Up,
// Average, Paeth) whose output has the smallest sum of |signed bytes| (the
// first of equal sums).  Each filter is its own branch-free loop over the
// row (the compiler vectorises them): five sums, then the chosen filter once.
// a = the byte 3 to the left (0 in the first pixel), b = above, c = above-left
template <int F>
inline uint8_t fpred(int a, int b, int c) {
  if constexpr (F == 1) return static_cast<uint8_t>(a);
  else if constexpr (F == 2) return static_cast<uint8_t>(b);
  else if constexpr (F == 3) return static_cast<uint8_t>((a + b) >> 1);
  else if constexpr (F == 4) {
    const int pa = std::abs(b - c), pb = std::abs(a - c), pc = std::abs(a + b - 2 * c);
    return static_cast<uint8_t>((pa <= pb && pa <= pc) ? a : (pb <= pc ? b : c));
  } else {
    return 0;
  }
}

template <int F>
long filter_sum(const uint8_t* cur, const uint8_t* up, size_t stride) {
  long sum = 0;
  const size_t h = std::min<size_t>(3, stride);
  for (size_t i = 0; i < h; ++i) sum += std::abs(static_cast<int>(static_cast<int8_t>(cur[i] - fpred<F>(0, up[i], 0))));
  for (size_t i = 3; i < stride; ++i)
    sum += std::abs(static_cast<int>(static_cast<int8_t>(cur[i] - fpred<F>(cur[i - 3], up[i], up[i - 3]))));
  return sum;
}

template <int F>
void filter_apply(const uint8_t* cur, const uint8_t* up, size_t stride, uint8_t* o) {
  const size_t h = std::min<size_t>(3, stride);
  for (size_t i = 0; i < h; ++i) o[i] = static_cast<uint8_t>(cur[i] - fpred<F>(0, up[i], 0));
  for (size_t i = 3; i < stride; ++i) o[i] = static_cast<uint8_t>(cur[i] - fpred<F>(cur[i - 3], up[i], up[i - 3]));
}

void filter_row(const uint8_t* cur, const uint8_t* up, size_t stride, uint8_t* o) {
  const long sums[5] = {filter_sum<0>(cur, up, stride), filter_sum<1>(cur, up, stride),
                        filter_sum<2>(cur, up, stride), filter_sum<3>(cur, up, stride),
                        filter_sum<4>(cur, up, stride)};
  int best = 0;
  for (int f = 1; f < 5; ++f)
    if (sums[f] < sums[best]) best = f;
  o[0] = static_cast<uint8_t>(best);
  switch (best) {
    case 0: filter_apply<0>(cur, up, stride, o + 1); break;
    case 1: filter_apply<1>(cur, up, stride, o + 1); break;
    case 2: filter_apply<2>(cur, up, stride, o + 1); break;
    case 3: filter_apply<3>(cur, up, stride, o + 1); break;
    default: filter_apply<4>(cur, up, stride, o + 1); break;
  }
}

// host threads for the filter and deflate passes (a frame is independent
// rows and independently deflated chunks)
int png_threads() {
  const unsigned hc = std::thread::hardware_concurrency();
  return static_cast<int>(std::max(1u, std::min(16u, hc ? hc : 1u)));
}

template <class F>
void parallel_for(int n, F f) {
  const int nt = std::min(n, png_threads());
  if (nt <= 1) {
    for (int i = 0; i < n; ++i) f(i);
    return;
  }
  std::atomic<int> next{0};
  std::vector<std::thread> th;
  for (int t = 0; t < nt; ++t)
    th.emplace_back([&] {
      for (int i; (i = next.fetch_add(1)) < n;) f(i);
    });
  for (auto& x : th) x.join();
}

std::vector<uint8_t> filter_rows(const uint8_t* rgb, int w, int h) {
  const size_t stride = static_cast<size_t>(w) * 3;
  std::vector<uint8_t> out((stride + 1) * static_cast<size_t>(h));
  std::vector<uint8_t> zero(stride, 0);
  constexpr int kRowsPerTask = 16;
  parallel_for((h + kRowsPerTask - 1) / kRowsPerTask, [&](int task) {
    for (int y = task * kRowsPerTask; y < std::min(h, (task + 1) * kRowsPerTask); ++y)
      filter_row(rgb + stride * y, y > 0 ? rgb + stride * (y - 1) : zero.data(), stride,
                 out.data() + (stride + 1) * y);
  });
  return out;
}

// One zlib stream from independently deflated fixed-size chunks (the
// output does not depend on the thread count): each chunk a raw deflate run
// ended by a sync flush (byte-aligned, not final) -- the last one finished --
// behind the zlib header, then the Adler-32 of the whole input combined from
// the chunks'.  Valid for any inflater (RFC 1950/1951).  The IDAT chunk's
// CRC-32 is combined the same way from the parts' CRCs, each computed by the
// thread that deflated the part; nothing is copied into one buffer.
struct ZStream {
  std::vector<std::vector<uint8_t>> part;
  uint8_t trailer[4];
  size_t size = 0;      // zlib header + parts + trailer
  uLong idat_crc = 0;   // CRC-32 over "IDAT" and the whole stream
};

constexpr uint8_t kZlibHeader[2] = {0x78, 0x9c};

bool deflate_chunked(const std::vector<uint8_t>& raw, ZStream* z) {
  constexpr size_t kChunk = 64 * 1024;   // (deflate's window is 32 KB: chunks this size lose little)
  const size_t n = raw.size();
  const int nchunk = static_cast<int>(std::max<size_t>(1, (n + kChunk - 1) / kChunk));
  z->part.assign(nchunk, {});
  std::vector<uLong> adl(nchunk), crc(nchunk);
  std::atomic<bool> ok{true};
  parallel_for(nchunk, [&](int c) {
    const size_t b = static_cast<size_t>(c) * kChunk, len = std::min(kChunk, n - b);
    z_stream zs{};
    // Z_RLE (runs of the filtered bytes, then Huffman codes): C1's rendered
    // frame in 28 ms of one core against 50 for level 1's LZ77 and 203 for
    // level 6, and 996 KB against 1,065 / 991 (tools/png_stages.cpp; the
    // bytes are a lossless encoding either way, the pixels are the PPM's)
    if (deflateInit2(&zs, 1, Z_DEFLATED, -15, 8, Z_RLE) != Z_OK) {
      ok = false;
      return;
    }
    std::vector<uint8_t>& o = z->part[c];
    o.resize(deflateBound(&zs, static_cast<uLong>(len)) + 16);
    zs.next_in = const_cast<Bytef*>(raw.data() + b);
    zs.avail_in = static_cast<uInt>(len);
    zs.next_out = o.data();
    zs.avail_out = static_cast<uInt>(o.size());
    const int rc = deflate(&zs, c == nchunk - 1 ? Z_FINISH : Z_SYNC_FLUSH);
    if (rc != (c == nchunk - 1 ? Z_STREAM_END : Z_OK) || zs.avail_in != 0) ok = false;
    o.resize(o.size() - zs.avail_out);
    deflateEnd(&zs);
    adl[c] = adler32(adler32(0L, Z_NULL, 0), raw.data() + b, static_cast<uInt>(len));
    crc[c] = crc32(crc32(0L, Z_NULL, 0), o.data(), static_cast<uInt>(o.size()));
  });
  if (!ok) return false;
  uLong a = adl[0];
  for (int c = 1; c < nchunk; ++c)
    a = adler32_combine(a, adl[c], static_cast<z_off_t>(std::min(kChunk, n - static_cast<size_t>(c) * kChunk)));
  for (int k = 0; k < 4; ++k) z->trailer[k] = static_cast<uint8_t>(a >> (24 - 8 * k));
  uLong cr = crc32(crc32(0L, Z_NULL, 0), reinterpret_cast<const Bytef*>("IDAT"), 4);
  cr = crc32(cr, kZlibHeader, 2);
  z->size = 2 + 4;
  for (int c = 0; c < nchunk; ++c) {
    cr = crc32_combine(cr, crc[c], static_cast<z_off_t>(z->part[c].size()));
    z->size += z->part[c].size();
  }
  z->idat_crc = crc32(cr, z->trailer, 4);
  return true;
}

}  // namespace

extern "C" int rt_write_png(const char* path, const uint8_t* rgb, int width, int height) {
  rtclj::clear_error();
  if (!path || !rgb || width <= 0 || height <= 0)
    return rtclj::set_error(RT_E_ARG, "rt_write_png: bad argument");
  const std::vector<uint8_t> raw = filter_rows(rgb, width, height);
  ZStream z;
  if (!deflate_chunked(raw, &z) || z.size > 0x7fffffffu) return rtclj::set_error(RT_E_IO, "rt_write_png: deflate failed");
  // signature, IHDR, the IDAT chunk's length and type and zlib header; the
  // parts are written straight from their buffers, then the Adler-32, the
  // CRC and IEND
  std::vector<uint8_t> head = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
  std::vector<uint8_t> ihdr;
  put_u32(ihdr, static_cast<uint32_t>(width));
  put_u32(ihdr, static_cast<uint32_t>(height));
  ihdr.insert(ihdr.end(), {8, 2, 0, 0, 0});   // 8-bit, truecolour RGB, deflate, adaptive filters, no interlace
  chunk(head, "IHDR", ihdr.data(), ihdr.size());
  put_u32(head, static_cast<uint32_t>(z.size));
  head.insert(head.end(), {'I', 'D', 'A', 'T', kZlibHeader[0], kZlibHeader[1]});
  std::vector<uint8_t> tail(z.trailer, z.trailer + 4);
  put_u32(tail, static_cast<uint32_t>(z.idat_crc));
  chunk(tail, "IEND", nullptr, 0);
  FILE* f = std::fopen(path, "wb");
  if (!f) return rtclj::set_error(RT_E_IO, std::string("rt_write_png: cannot open ") + path);
  bool ok = std::fwrite(head.data(), 1, head.size(), f) == head.size();
  for (const auto& p : z.part) ok = ok && std::fwrite(p.data(), 1, p.size(), f) == p.size();
  ok = ok && std::fwrite(tail.data(), 1, tail.size(), f) == tail.size();
  ok = (std::fclose(f) == 0) && ok;
  if (!ok) return rtclj::set_error(RT_E_IO, std::string("rt_write_png: write failed: ") + path);
  return RT_OK;
}

// P3 -> PNG as ppm2png.clj:35-87: header "P3", "width height", a maximum
// colour value in [0, 255], then width*height pixels of three values (the
// reference reads one pixel per line; any whitespace is accepted here).
// Values are written as they are (ppm2png packs r<<16|g<<8|b unscaled).
// The pixel values (2.4 M numbers, 9 MB of text in a C1 frame) are parsed in parallel:
// the text is cut at whitespace into one span per thread, each span's values
// parsed into its own buffer, then placed by the spans' counts; an error is
// the first one in text order, reported at its pixel as a sequential parse
// would, and text beyond the last pixel is ignored as before.
namespace {

bool is_space(char ch) { return ch == ' ' || ch == '\n' || ch == '\r' || ch == '\t' || ch == '\v' || ch == '\f'; }

// a whitespace-delimited decimal of at most 9 digits at t[*pos] (after
// whitespace); false on anything else.  end is the span's end: a whitespace
// character or the text's end
bool parse_number(const char* t, size_t end, size_t* pos, long* v) {
  size_t p = *pos;
  while (p < end && is_space(t[p])) ++p;
  const size_t b = p;
  long x = 0;
  // (a tenth digit ends the parse before it is multiplied in: no overflow)
  while (p < end && t[p] >= '0' && t[p] <= '9') {
    if (p - b == 9) return false;
    x = x * 10 + (t[p++] - '0');
  }
  *pos = p;
  if (p == b || (p < end && !is_space(t[p]))) return false;
  *v = x;
  return true;
}

struct Span {
  std::vector<uint8_t> v;   // the span's values, in order
  bool bad = false;         // stopped at a token that is no value (or above the maximum)
};

}  // namespace

extern "C" int rt_ppm_to_png(const char* src, const char* dst) {
  rtclj::clear_error();
  if (!src || !dst) return rtclj::set_error(RT_E_ARG, "rt_ppm_to_png: NULL path");
  FILE* f = std::fopen(src, "rb");
  if (!f) return rtclj::set_error(RT_E_IO, std::string("rt_ppm_to_png: cannot open ") + src);
  std::string text;
  long sz = -1;
  if (std::fseek(f, 0, SEEK_END) == 0) {   // (one read straight into the text where the size is known)
    sz = std::ftell(f);
    if (std::fseek(f, 0, SEEK_SET) != 0) sz = -1;
  }
  if (sz > 0) {
    text.resize(static_cast<size_t>(sz));
    text.resize(std::fread(&text[0], 1, text.size(), f));
  }
  char buf[1 << 16];   // (the rest, or a stream of unknown size)
  for (size_t n; (n = std::fread(buf, 1, sizeof buf, f)) > 0;) text.append(buf, n);
  std::fclose(f);
  size_t pos = 0;
  const char* t = text.data();
  const size_t tn = text.size();
  while (pos < tn && is_space(t[pos])) ++pos;
  if (!(pos + 2 <= tn && t[pos] == 'P' && t[pos + 1] == '3' && (pos + 2 == tn || is_space(t[pos + 2]))))
    return rtclj::set_error(RT_E_ARG, std::string("rt_ppm_to_png: ") + src + ": bad header");
  pos += 2;
  long w = 0, h = 0, maxv = 0;
  if (!parse_number(t, tn, &pos, &w) || !parse_number(t, tn, &pos, &h) || w <= 0 || h <= 0 || w > 65535 || h > 65535)
    return rtclj::set_error(RT_E_ARG, std::string("rt_ppm_to_png: ") + src + ": bad dimensions");
  if (!parse_number(t, tn, &pos, &maxv) || maxv > 255)
    return rtclj::set_error(RT_E_ARG, std::string("rt_ppm_to_png: ") + src + ": bad colour size");
  const size_t need = static_cast<size_t>(w) * h * 3;
  // spans of ~256 KB (at least one, at most 256), cut at whitespace so no
  // token is split
  const size_t body = tn - pos;
  const int nspan = static_cast<int>(std::max<size_t>(1, std::min<size_t>(256, body >> 18)));
  std::vector<size_t> cut(nspan + 1);
  cut[0] = pos;
  cut[nspan] = tn;
  for (int k = 1; k < nspan; ++k) {
    size_t c = std::max(cut[k - 1], pos + body / nspan * k);
    while (c < tn && !is_space(t[c])) ++c;
    cut[k] = c;
  }
  std::vector<Span> span(nspan);
  parallel_for(nspan, [&](int k) {
    Span& s = span[k];
    s.v.reserve((cut[k + 1] - cut[k]) / 3 + 16);
    size_t p = cut[k];
    const size_t end = cut[k + 1];
    for (;;) {
      while (p < end && is_space(t[p])) ++p;
      if (p == end) break;
      long v = 0;
      if (!parse_number(t, end, &p, &v) || v > maxv) {
        s.bad = true;
        break;
      }
      s.v.push_back(static_cast<uint8_t>(v));
    }
  });
  std::vector<uint8_t> rgb(need);
  size_t got = 0;
  for (int k = 0; k < nspan && got < need; ++k) {
    const size_t take = std::min(span[k].v.size(), need - got);
    std::memcpy(rgb.data() + got, span[k].v.data(), take);
    got += take;
    if (got < need && span[k].bad) break;   // the first bad token before the last pixel
  }
  if (got < need)
    return rtclj::set_error(RT_E_ARG, std::string("rt_ppm_to_png: ") + src + ": bad pixel value at " +
                                          std::to_string(got / 3));
  return rt_write_png(dst, rgb.data(), static_cast<int>(w), static_cast<int>(h));
}
