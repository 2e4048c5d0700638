// png_io.hpp — PNG codec on zlib for the CLI: texture decode with the
// reference's RMagick view (every sample as a 16-bit quantum, `>> 8` kept:
// src/objects/texture.rb:12-20) and RGBA8 encode of the canvas
// (Camera#save_image, src/camera.rb:36-39).  Same conventions as
// raytracing_rb_amd/png.py, which the tests compare it with.
#pragma once

#include <zlib.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <stdexcept>
#include <string>
#include <vector>

namespace rtxcli {

inline uint32_t be32(const uint8_t* p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }

inline std::vector<uint8_t> read_file(const std::string& path) {
  FILE* f = fopen(path.c_str(), "rb");
  if (!f) throw std::runtime_error("cannot open " + path);
  std::vector<uint8_t> d;
  uint8_t buf[65536];
  size_t n;
  while ((n = fread(buf, 1, sizeof buf, f)) > 0) d.insert(d.end(), buf, buf + n);
  fclose(f);
  return d;
}

// Decode to RGB8 rows top-down (H x W x 3).
inline std::vector<uint8_t> png_decode_rgb8(const std::string& path, int& w, int& h) {
  const std::vector<uint8_t> d = read_file(path);
  static const uint8_t sig[8] = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
  if (d.size() < 8 || !std::equal(sig, sig + 8, d.begin())) throw std::runtime_error(path + ": not a PNG file");
  size_t pos = 8;
  int depth = 0, ctype = 0, interlace = 0;
  w = h = 0;
  std::vector<uint8_t> idat, plte;
  while (pos + 8 <= d.size()) {
    const uint32_t n = be32(&d[pos]);
    const std::string tag(d.begin() + pos + 4, d.begin() + pos + 8);
    if (pos + 12 + n > d.size()) throw std::runtime_error(path + ": truncated chunk");
    const uint8_t* body = &d[pos + 8];
    if (tag == "IHDR") {
      w = (int)be32(body);
      h = (int)be32(body + 4);
      depth = body[8];
      ctype = body[9];
      interlace = body[12];
    } else if (tag == "PLTE") {
      plte.assign(body, body + n);
    } else if (tag == "IDAT") {
      idat.insert(idat.end(), body, body + n);
    } else if (tag == "IEND") {
      break;
    }
    pos += 12 + n;
  }
  if (interlace) throw std::runtime_error(path + ": interlaced PNG not supported");
  int chans;
  switch (ctype) {
    case 0: chans = 1; break;
    case 2: chans = 3; break;
    case 3: chans = 1; break;
    case 4: chans = 2; break;
    case 6: chans = 4; break;
    default: throw std::runtime_error(path + ": bad color type");
  }
  const int bits = depth * chans;
  const int bpp = bits / 8 > 0 ? bits / 8 : 1;
  const size_t stride = ((size_t)w * bits + 7) / 8;
  std::vector<uint8_t> raw((stride + 1) * h);
  uLongf rlen = raw.size();
  if (uncompress(raw.data(), &rlen, idat.data(), idat.size()) != Z_OK || rlen != raw.size())
    throw std::runtime_error(path + ": bad image data");
  std::vector<uint8_t> img(stride * h), prev(stride, 0);
  for (int y = 0; y < h; y++) {
    const uint8_t ft = raw[y * (stride + 1)];
    uint8_t* line = &img[y * stride];
    const uint8_t* src = &raw[y * (stride + 1) + 1];
    for (size_t i = 0; i < stride; i++) {
      const int a = i >= (size_t)bpp ? line[i - bpp] : 0;
      const int b = prev[i];
      const int c = i >= (size_t)bpp ? prev[i - bpp] : 0;
      int v = src[i];
      if (ft == 1) v += a;
      else if (ft == 2) v += b;
      else if (ft == 3) v += (a + b) >> 1;
      else if (ft == 4) {
        const int p = a + b - c, pa = abs(p - a), pb = abs(p - b), pc = abs(p - c);
        v += (pa <= pb && pa <= pc) ? a : (pb <= pc ? b : c);
      } else if (ft != 0) {
        throw std::runtime_error(path + ": bad filter type");
      }
      line[i] = (uint8_t)v;
    }
    std::copy(line, line + stride, prev.begin());
  }
  std::vector<uint8_t> out((size_t)w * h * 3);
  for (int y = 0; y < h; y++)
    for (int x = 0; x < w; x++) {
      int s[4] = {0, 0, 0, 0};
      for (int c = 0; c < chans; c++) {
        if (depth == 16) s[c] = img[y * stride + ((size_t)x * chans + c) * 2];             // high byte (>> 8)
        else if (depth == 8) s[c] = img[y * stride + (size_t)x * chans + c];
        else {                                                                        // 1/2/4-bit
          const size_t bit = (size_t)x * depth;
          const int v = (img[y * stride + bit / 8] >> (8 - depth - (int)(bit % 8))) & ((1 << depth) - 1);
          s[c] = ctype == 0 ? v * (255 / ((1 << depth) - 1)) : v;
        }
      }
      uint8_t* o = &out[((size_t)y * w + x) * 3];
      if (ctype == 3) {
        if ((size_t)s[0] * 3 + 2 >= plte.size()) throw std::runtime_error(path + ": palette index out of range");
        o[0] = plte[s[0] * 3];
        o[1] = plte[s[0] * 3 + 1];
        o[2] = plte[s[0] * 3 + 2];
      } else if (chans <= 2) {
        o[0] = o[1] = o[2] = (uint8_t)s[0];
      } else {
        o[0] = (uint8_t)s[0];
        o[1] = (uint8_t)s[1];
        o[2] = (uint8_t)s[2];
      }
    }
  return out;
}

inline void put_chunk(std::vector<uint8_t>& o, const char* tag, const std::vector<uint8_t>& body) {
  const uint32_t n = (uint32_t)body.size();
  const uint8_t len[4] = {(uint8_t)(n >> 24), (uint8_t)(n >> 16), (uint8_t)(n >> 8), (uint8_t)n};
  o.insert(o.end(), len, len + 4);
  const size_t start = o.size();
  o.insert(o.end(), tag, tag + 4);
  o.insert(o.end(), body.begin(), body.end());
  const uint32_t crc = (uint32_t)crc32(0, &o[start], (uInt)(o.size() - start));
  const uint8_t c[4] = {(uint8_t)(crc >> 24), (uint8_t)(crc >> 16), (uint8_t)(crc >> 8), (uint8_t)crc};
  o.insert(o.end(), c, c + 4);
}

// Encode H x W x 4 RGBA8 rows top-down (zlib level 6, filter 0 — the bytes
// png.py writes).
inline void png_write_rgba8(const std::string& path, const uint8_t* rgba, int w, int h) {
  std::vector<uint8_t> raw;
  raw.reserve(((size_t)w * 4 + 1) * h);
  for (int y = 0; y < h; y++) {
    raw.push_back(0);
    raw.insert(raw.end(), rgba + (size_t)y * w * 4, rgba + (size_t)(y + 1) * w * 4);
  }
  uLongf zlen = compressBound(raw.size());
  std::vector<uint8_t> z(zlen);
  if (compress2(z.data(), &zlen, raw.data(), raw.size(), 6) != Z_OK) throw std::runtime_error("zlib failed");
  z.resize(zlen);
  std::vector<uint8_t> o = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
  std::vector<uint8_t> ihdr = {(uint8_t)(w >> 24), (uint8_t)(w >> 16), (uint8_t)(w >> 8), (uint8_t)w,
                               (uint8_t)(h >> 24), (uint8_t)(h >> 16), (uint8_t)(h >> 8), (uint8_t)h,
                               8, 6, 0, 0, 0};
  put_chunk(o, "IHDR", ihdr);
  put_chunk(o, "IDAT", z);
  put_chunk(o, "IEND", {});
  FILE* f = fopen(path.c_str(), "wb");
  if (!f) throw std::runtime_error("cannot write " + path);
  const bool ok = fwrite(o.data(), 1, o.size(), f) == o.size();
  if (fclose(f) != 0 || !ok) throw std::runtime_error("cannot write " + path);
}

}  // namespace rtxcli
