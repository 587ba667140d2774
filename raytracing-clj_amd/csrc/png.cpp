// png.cpp — PNG output for the host side: rt_write_png (8-bit RGB from the
// quantised frame) and rt_ppm_to_png, the behaviour of the reference's
// src/ppm2png.clj:35-87 (P3 in, 8-bit RGB PNG out).  Written from the PNG
// specification (signature, IHDR / IDAT / IEND chunks with CRC-32, zlib
// stream of per-row filtered scanlines); deflate and CRC come from zlib.
#include <zlib.h>

#include <cctype>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
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
std::vector<uint8_t> filter_rows(const uint8_t* rgb, int w, int h) {
  const size_t stride = static_cast<size_t>(w) * 3;
  std::vector<uint8_t> out((stride + 1) * static_cast<size_t>(h));
  std::vector<uint8_t> cand[5];
  for (auto& c : cand) c.resize(stride);
  std::vector<uint8_t> zero(stride, 0);
  for (int y = 0; y < h; ++y) {
    const uint8_t* cur = rgb + stride * y;
    const uint8_t* up = y > 0 ? rgb + stride * (y - 1) : zero.data();
    long best_sum = -1;
    int best = 0;
    for (int f = 0; f < 5; ++f) {
      long sum = 0;
      for (size_t i = 0; i < stride; ++i) {
        const int a = i >= 3 ? cur[i - 3] : 0, b = up[i], c = i >= 3 ? up[i - 3] : 0;
        int pred = 0;
        switch (f) {
          case 1: pred = a; break;
          case 2: pred = b; break;
          case 3: pred = (a + b) >> 1; break;
          case 4: pred = paeth(a, b, c); break;
          default: break;
        }
        const uint8_t v = static_cast<uint8_t>(cur[i] - pred);
        cand[f][i] = v;
        sum += v < 128 ? v : 256 - v;
      }
      if (best_sum < 0 || sum < best_sum) {
        best_sum = sum;
        best = f;
      }
    }
    uint8_t* o = out.data() + (stride + 1) * y;
    o[0] = static_cast<uint8_t>(best);
    std::memcpy(o + 1, cand[best].data(), stride);
  }
  return out;
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
  uLongf zlen = compressBound(static_cast<uLong>(raw.size()));
  std::vector<uint8_t> z(zlen);
  if (compress2(z.data(), &zlen, raw.data(), static_cast<uLong>(raw.size()), 6) != Z_OK || zlen > 0x7fffffffu)
    return rtclj::set_error(RT_E_IO, "rt_write_png: deflate failed");
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
  size_t pos = 0;
  auto token = [&](std::string* out) {
    while (pos < text.size() && std::isspace(static_cast<unsigned char>(text[pos]))) ++pos;
    const size_t b = pos;
    while (pos < text.size() && !std::isspace(static_cast<unsigned char>(text[pos]))) ++pos;
    out->assign(text, b, pos - b);
    return pos > b;
  };
  auto number = [&](long* v) {
    std::string t;
    if (!token(&t) || t.empty() || t.size() > 9) return false;
    for (char ch : t)
      if (!std::isdigit(static_cast<unsigned char>(ch))) return false;
    *v = std::strtol(t.c_str(), nullptr, 10);
    return true;
  };
  std::string magic;
  if (!token(&magic) || magic != "P3")
    return rtclj::set_error(RT_E_ARG, std::string("rt_ppm_to_png: ") + src + ": bad header");
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
