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

int paeth(int a, int b, int c) {
  const int p = a + b - c;
  const int pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - c);
  if (pa <= pb && pa <= pc) return a;
  return pb <= pc ? b : c;
}

// scanlines with a filter byte each; per row the filter (None, Sub, Up,
// Average, Paeth) whose output has the smallest sum of |signed bytes|
void filter_row(const uint8_t* cur, const uint8_t* up, size_t stride, uint8_t* o, uint8_t* tmp) {
  long best_sum = -1;
  int best = 0;
  for (int f = 0; f < 5; ++f) {
    long sum = 0;
    uint8_t* c = f == 0 ? o + 1 : tmp;   // (None first, straight into the output row)
    for (size_t i = 0; i < stride; ++i) {
      const int a = i >= 3 ? cur[i - 3] : 0, b = up[i], cc = i >= 3 ? up[i - 3] : 0;
      int pred = 0;
      switch (f) {
        case 1: pred = a; break;
        case 2: pred = b; break;
        case 3: pred = (a + b) >> 1; break;
        case 4: pred = paeth(a, b, cc); break;
        default: break;
      }
      const uint8_t v = static_cast<uint8_t>(cur[i] - pred);
      c[i] = v;
      sum += v < 128 ? v : 256 - v;
    }
    if (best_sum < 0 || sum < best_sum) {
      best_sum = sum;
      best = f;
      if (f > 0) std::memcpy(o + 1, tmp, stride);
    }
  }
  o[0] = static_cast<uint8_t>(best);
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
  constexpr int kRowsPerTask = 32;
  parallel_for((h + kRowsPerTask - 1) / kRowsPerTask, [&](int task) {
    std::vector<uint8_t> tmp(stride);
    for (int y = task * kRowsPerTask; y < std::min(h, (task + 1) * kRowsPerTask); ++y)
      filter_row(rgb + stride * y, y > 0 ? rgb + stride * (y - 1) : zero.data(), stride,
                 out.data() + (stride + 1) * y, tmp.data());
  });
  return out;
}

// One zlib stream from independently deflated fixed-size chunks (the
// output does not depend on the thread count): each chunk a raw deflate run
// ended by a sync flush (byte-aligned, not final) -- the last one finished --
// behind the zlib header, then the Adler-32 of the whole input combined from
// the chunks'.  Valid for any inflater (RFC 1950/1951).
bool deflate_chunked(const std::vector<uint8_t>& raw, std::vector<uint8_t>* z) {
  constexpr size_t kChunk = 256 * 1024;
  const size_t n = raw.size();
  const int nchunk = static_cast<int>(std::max<size_t>(1, (n + kChunk - 1) / kChunk));
  std::vector<std::vector<uint8_t>> part(nchunk);
  std::vector<uLong> adl(nchunk);
  std::atomic<bool> ok{true};
  parallel_for(nchunk, [&](int c) {
    const size_t b = static_cast<size_t>(c) * kChunk, len = std::min(kChunk, n - b);
    z_stream zs{};
    // level 1: a C1 frame in ~1/2.5 of level 6's time for a 13 % larger file
    // (the bytes are a lossless encoding either way; the pixels are the PPM's)
    if (deflateInit2(&zs, 1, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY) != Z_OK) {
      ok = false;
      return;
    }
    std::vector<uint8_t>& o = part[c];
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
  });
  if (!ok) return false;
  z->assign({0x78, 0x9c});
  uLong a = adl[0];
  for (int c = 0; c < nchunk; ++c) {
    z->insert(z->end(), part[c].begin(), part[c].end());
    if (c > 0) a = adler32_combine(a, adl[c], static_cast<z_off_t>(std::min(kChunk, n - static_cast<size_t>(c) * kChunk)));
  }
  put_u32(*z, static_cast<uint32_t>(a));
  return true;
}

int write_file(const char* path, const std::vector<uint8_t>& bytes, const char* who) {
  FILE* f = std::fopen(path, "wb");
  if (!f) return rtclj::set_error(RT_E_IO, std::string(who) + ": cannot open " + path);
  const size_t n = std::fwrite(bytes.data(), 1, bytes.size(), f);
  const bool ok = n == bytes.size() && std::fclose(f) == 0;
  if (!ok) return rtclj::set_error(RT_E_IO, std::string(who) + ": write failed: " + path);
  return RT_OK;
}

}  // namespace

extern "C" int rt_write_png(const char* path, const uint8_t* rgb, int width, int height) {
  rtclj::clear_error();
  if (!path || !rgb || width <= 0 || height <= 0)
    return rtclj::set_error(RT_E_ARG, "rt_write_png: bad argument");
  const std::vector<uint8_t> raw = filter_rows(rgb, width, height);
  std::vector<uint8_t> z;
  if (!deflate_chunked(raw, &z) || z.size() > 0x7fffffffu) return rtclj::set_error(RT_E_IO, "rt_write_png: deflate failed");
  const size_t zlen = z.size();
  std::vector<uint8_t> png = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
  std::vector<uint8_t> ihdr;
  put_u32(ihdr, static_cast<uint32_t>(width));
  put_u32(ihdr, static_cast<uint32_t>(height));
  ihdr.insert(ihdr.end(), {8, 2, 0, 0, 0});   // 8-bit, truecolour RGB, deflate, adaptive filters, no interlace
  chunk(png, "IHDR", ihdr.data(), ihdr.size());
  chunk(png, "IDAT", z.data(), zlen);
  chunk(png, "IEND", nullptr, 0);
  return write_file(path, png, "rt_write_png");
}

// P3 -> PNG as ppm2png.clj:35-87: header "P3", "width height", a maximum
// colour value in [0, 255], then width*height pixels of three values (the
// reference reads one pixel per line; any whitespace is accepted here).
// Values are written as they are (ppm2png packs r<<16|g<<8|b unscaled).
extern "C" int rt_ppm_to_png(const char* src, const char* dst) {
  rtclj::clear_error();
  if (!src || !dst) return rtclj::set_error(RT_E_ARG, "rt_ppm_to_png: NULL path");
  FILE* f = std::fopen(src, "rb");
  if (!f) return rtclj::set_error(RT_E_IO, std::string("rt_ppm_to_png: cannot open ") + src);
  std::string text;
  char buf[1 << 16];
  for (size_t n; (n = std::fread(buf, 1, sizeof buf, f)) > 0;) text.append(buf, n);
  std::fclose(f);
  // (a hand-rolled scan: 2.4 M numbers in a C1 frame)
  size_t pos = 0;
  const char* t = text.data();
  const size_t tn = text.size();
  auto space = [](char ch) { return ch == ' ' || ch == '\n' || ch == '\r' || ch == '\t' || ch == '\v' || ch == '\f'; };
  auto skip = [&] {
    while (pos < tn && space(t[pos])) ++pos;
  };
  // a whitespace-delimited decimal of at most 9 digits; false on anything else
  auto number = [&](long* v) {
    skip();
    const size_t b = pos;
    long x = 0;
    // (a tenth digit ends the parse before it is multiplied in: no overflow)
    while (pos < tn && t[pos] >= '0' && t[pos] <= '9') {
      if (pos - b == 9) return false;
      x = x * 10 + (t[pos++] - '0');
    }
    if (pos == b || (pos < tn && !space(t[pos]))) return false;
    *v = x;
    return true;
  };
  skip();
  if (!(pos + 2 <= tn && t[pos] == 'P' && t[pos + 1] == '3' && (pos + 2 == tn || space(t[pos + 2]))))
    return rtclj::set_error(RT_E_ARG, std::string("rt_ppm_to_png: ") + src + ": bad header");
  pos += 2;
  long w = 0, h = 0, maxv = 0;
  if (!number(&w) || !number(&h) || w <= 0 || h <= 0 || w > 65535 || h > 65535)
    return rtclj::set_error(RT_E_ARG, std::string("rt_ppm_to_png: ") + src + ": bad dimensions");
  if (!number(&maxv) || maxv > 255)
    return rtclj::set_error(RT_E_ARG, std::string("rt_ppm_to_png: ") + src + ": bad colour size");
  std::vector<uint8_t> rgb(static_cast<size_t>(w) * h * 3);
  for (size_t i = 0; i < rgb.size(); ++i) {
    long v = 0;
    if (!number(&v) || v > maxv)
      return rtclj::set_error(RT_E_ARG, std::string("rt_ppm_to_png: ") + src + ": bad pixel value at " +
                                            std::to_string(i / 3));
    rgb[i] = static_cast<uint8_t>(v);
  }
  return rt_write_png(dst, rgb.data(), static_cast<int>(w), static_cast<int>(h));
}
