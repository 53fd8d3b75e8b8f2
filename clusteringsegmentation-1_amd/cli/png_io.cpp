// png_io.cpp -- see png_io.h.
#include "png_io.h"

#include <zlib.h>

#include <algorithm>
#include <cstdio>
#include <cstring>

namespace dqcli {

namespace {

uint32_t be32(const uint8_t* p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

void put_be32(std::vector<uint8_t>& v, uint32_t x) {
  v.push_back((uint8_t)(x >> 24));
  v.push_back((uint8_t)(x >> 16));
  v.push_back((uint8_t)(x >> 8));
  v.push_back((uint8_t)x);
}

const uint8_t kSig[8] = {137, 80, 78, 71, 13, 10, 26, 10};

bool fail(std::string* err, const std::string& why) {
  if (err) *err = why;
  return false;
}

uint8_t paeth(int a, int b, int c) {
  const int p = a + b - c;
  const int pa = p > a ? p - a : a - p, pb = p > b ? p - b : b - p, pc = p > c ? p - c : c - p;
  if (pa <= pb && pa <= pc) return (uint8_t)a;
  if (pb <= pc) return (uint8_t)b;
  return (uint8_t)c;
}

}  // namespace

bool read_png_bgr(const std::string& path, Image* img, std::string* err) {
  FILE* f = std::fopen(path.c_str(), "rb");
  if (!f) return fail(err, "cannot open");
  std::vector<uint8_t> file;
  {
    uint8_t buf[1 << 16];
    size_t n;
    while ((n = std::fread(buf, 1, sizeof buf, f)) > 0) file.insert(file.end(), buf, buf + n);
    std::fclose(f);
  }
  if (file.size() < 8 || std::memcmp(file.data(), kSig, 8) != 0) return fail(err, "not a PNG file");
  uint32_t w = 0, h = 0;
  int depth = 0, ctype = -1, interlace = 0;
  std::vector<uint8_t> plte, idat;
  size_t pos = 8;
  bool ended = false;
  while (pos + 12 <= file.size() && !ended) {
    const uint32_t len = be32(&file[pos]);
    if (pos + 12 + (size_t)len > file.size()) return fail(err, "truncated chunk");
    const char* type = (const char*)&file[pos + 4];
    const uint8_t* data = &file[pos + 8];
    if (std::memcmp(type, "IHDR", 4) == 0) {
      if (len != 13) return fail(err, "bad IHDR");
      w = be32(data);
      h = be32(data + 4);
      depth = data[8];
      ctype = data[9];
      if (data[10] != 0 || data[11] != 0) return fail(err, "unknown compression or filter method");
      interlace = data[12];
    } else if (std::memcmp(type, "PLTE", 4) == 0) {
      plte.assign(data, data + len);
    } else if (std::memcmp(type, "IDAT", 4) == 0) {
      idat.insert(idat.end(), data, data + len);
    } else if (std::memcmp(type, "IEND", 4) == 0) {
      ended = true;
    }
    pos += 12 + (size_t)len;
  }
  if (w == 0 || h == 0 || ctype < 0) return fail(err, "missing IHDR");
  if (interlace != 0) return fail(err, "Adam7-interlaced PNGs are not supported");
  int chans;
  switch (ctype) {
    case 0: chans = 1; break;
    case 2: chans = 3; break;
    case 3: chans = 1; break;
    case 4: chans = 2; break;
    case 6: chans = 4; break;
    default: return fail(err, "unknown colour type");
  }
  const bool ok_depth = (ctype == 0 && (depth == 1 || depth == 2 || depth == 4 || depth == 8 || depth == 16)) ||
                        (ctype == 3 && (depth == 1 || depth == 2 || depth == 4 || depth == 8)) ||
                        ((ctype == 2 || ctype == 4 || ctype == 6) && (depth == 8 || depth == 16));
  if (!ok_depth) return fail(err, "invalid bit depth for the colour type");
  if (ctype == 3 && (plte.empty() || plte.size() % 3 != 0)) return fail(err, "missing PLTE");
  const size_t row_bytes = ((size_t)w * chans * depth + 7) / 8;
  const size_t bpp = std::max<size_t>(1, (size_t)chans * depth / 8);
  std::vector<uint8_t> raw((row_bytes + 1) * h);
  {
    z_stream zs;
    std::memset(&zs, 0, sizeof zs);
    if (inflateInit(&zs) != Z_OK) return fail(err, "zlib init");
    zs.next_in = idat.data();
    zs.avail_in = (uInt)idat.size();
    zs.next_out = raw.data();
    zs.avail_out = (uInt)raw.size();
    const int r = inflate(&zs, Z_FINISH);
    const size_t got = raw.size() - zs.avail_out;
    inflateEnd(&zs);
    if ((r != Z_STREAM_END && r != Z_OK && r != Z_BUF_ERROR) || got != raw.size())
      return fail(err, "corrupt image data");
  }
  // undo the per-row filters (in place; row y's bytes at raw[y*(rb+1)+1 ...])
  for (uint32_t y = 0; y < h; ++y) {
    uint8_t* row = &raw[(size_t)y * (row_bytes + 1)];
    const uint8_t ft = row[0];
    uint8_t* cur = row + 1;
    const uint8_t* prev = y ? &raw[(size_t)(y - 1) * (row_bytes + 1) + 1] : nullptr;
    for (size_t i = 0; i < row_bytes; ++i) {
      const int a = i >= bpp ? cur[i - bpp] : 0;
      const int b = prev ? prev[i] : 0;
      const int c = (prev && i >= bpp) ? prev[i - bpp] : 0;
      switch (ft) {
        case 0: break;
        case 1: cur[i] = (uint8_t)(cur[i] + a); break;
        case 2: cur[i] = (uint8_t)(cur[i] + b); break;
        case 3: cur[i] = (uint8_t)(cur[i] + ((a + b) >> 1)); break;
        case 4: cur[i] = (uint8_t)(cur[i] + paeth(a, b, c)); break;
        default: return fail(err, "unknown row filter");
      }
    }
  }
  img->width = w;
  img->height = h;
  img->bgr.assign((size_t)w * h * 3, 0);
  // sample s of a row (channel-interleaved), reduced to 8 bits as imread does
  auto sample = [&](const uint8_t* row, size_t s) -> uint32_t {
    if (depth == 8) return row[s];
    if (depth == 16) return row[2 * s];   // high byte (png_set_strip_16)
    const size_t bit = s * depth;
    const uint32_t v = (row[bit >> 3] >> (8 - depth - (bit & 7))) & ((1u << depth) - 1);
    return v;
  };
  for (uint32_t y = 0; y < h; ++y) {
    const uint8_t* row = &raw[(size_t)y * (row_bytes + 1) + 1];
    uint8_t* out = &img->bgr[(size_t)y * w * 3];
    for (uint32_t x = 0; x < w; ++x) {
      uint32_t r, g, b;
      if (ctype == 3) {
        const uint32_t idx = sample(row, x);
        if (3 * (size_t)idx + 2 >= plte.size()) return fail(err, "palette index out of range");
        r = plte[3 * idx];
        g = plte[3 * idx + 1];
        b = plte[3 * idx + 2];
      } else if (ctype == 0 || ctype == 4) {
        uint32_t v = sample(row, (size_t)x * chans);
        if (depth < 8) v = v * (255u / ((1u << depth) - 1));   // 1/2/4-bit grey expanded to 8 bits
        r = g = b = v;
      } else {
        r = sample(row, (size_t)x * chans);
        g = sample(row, (size_t)x * chans + 1);
        b = sample(row, (size_t)x * chans + 2);
      }
      out[3 * x] = (uint8_t)b;
      out[3 * x + 1] = (uint8_t)g;
      out[3 * x + 2] = (uint8_t)r;
    }
  }
  return true;
}

bool write_png_bgr(const std::string& path, const Image& img, std::string* err) {
  const uint32_t w = img.width, h = img.height;
  if (w == 0 || h == 0 || img.bgr.size() != (size_t)w * h * 3) return fail(err, "bad image");
  std::vector<uint8_t> raw(((size_t)w * 3 + 1) * h);
  for (uint32_t y = 0; y < h; ++y) {
    uint8_t* row = &raw[(size_t)y * (w * 3 + 1)];
    row[0] = 0;   // filter: none
    const uint8_t* in = &img.bgr[(size_t)y * w * 3];
    for (uint32_t x = 0; x < w; ++x) {
      row[1 + 3 * x] = in[3 * x + 2];
      row[2 + 3 * x] = in[3 * x + 1];
      row[3 + 3 * x] = in[3 * x];
    }
  }
  uLongf zlen = compressBound((uLong)raw.size());
  std::vector<uint8_t> z(zlen);
  if (compress2(z.data(), &zlen, raw.data(), (uLong)raw.size(), 6) != Z_OK) return fail(err, "zlib compress");
  z.resize(zlen);
  std::vector<uint8_t> out(kSig, kSig + 8);
  auto chunk = [&](const char* type, const std::vector<uint8_t>& data) {
    put_be32(out, (uint32_t)data.size());
    const size_t t0 = out.size();
    out.insert(out.end(), type, type + 4);
    out.insert(out.end(), data.begin(), data.end());
    put_be32(out, (uint32_t)crc32(0L, &out[t0], (uInt)(out.size() - t0)));
  };
  std::vector<uint8_t> ihdr;
  put_be32(ihdr, w);
  put_be32(ihdr, h);
  ihdr.insert(ihdr.end(), {8, 2, 0, 0, 0});   // 8-bit RGB, deflate, adaptive filters, no interlace
  chunk("IHDR", ihdr);
  chunk("IDAT", z);
  chunk("IEND", {});
  FILE* f = std::fopen(path.c_str(), "wb");
  if (!f) return fail(err, "cannot create");
  const bool ok = std::fwrite(out.data(), 1, out.size(), f) == out.size();
  return (std::fclose(f) == 0 && ok) ? true : fail(err, "write error");
}

}  // namespace dqcli
