// png.cpp -- host-side batched PNG encoder for the restored images
// (17_run_unified_inference.py:89-99: clamp -> x255 -> uint8 -> RGB2BGR ->
// cv2.imwrite per image).  cv2.imwrite of the BGR array stores the RGB
// pixels, so the file content is the RGB uint8 image: this writes it
// directly from the NHWC uint8 batch that rr_to_uint8_hwc produced.
//
// Format: 8-bit truecolour (c = 3) or greyscale (c = 1), no interlace, one
// IDAT from zlib (deflate level `level`); per-row filter chosen by the
// minimum-sum-of-absolute-differences heuristic over the five PNG filters
// (libpng's default adaptive choice).  Images are encoded on `threads`
// host threads (one file each); the GPU is not involved.
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "../../include/roadrestore.h"

namespace {

void put32(std::vector<uint8_t> &o, uint32_t v) {
  o.push_back(v >> 24); o.push_back((v >> 16) & 255); o.push_back((v >> 8) & 255); o.push_back(v & 255);
}

void chunk(std::vector<uint8_t> &o, const char *type, const uint8_t *data, size_t len) {
  put32(o, (uint32_t)len);
  const size_t t0 = o.size();
  o.insert(o.end(), type, type + 4);
  if (len) o.insert(o.end(), data, data + len);
  const uint32_t crc = (uint32_t)crc32(0L, o.data() + t0, (uInt)(len + 4));
  put32(o, crc);
}

inline uint8_t paeth(int a, int b, int c) {
  const int p = a + b - c, pa = abs(p - a), pb = abs(p - b), pc = abs(p - c);
  return (uint8_t)(pa <= pb && pa <= pc ? a : (pb <= pc ? b : c));
}

// filtered scanlines (filter byte + row) of one image
void filter_rows(int h, int w, int c, const uint8_t *img, std::vector<uint8_t> &out) {
  const size_t row = (size_t)w * c;
  out.resize((size_t)h * (row + 1));
  std::vector<uint8_t> cand[5];
  for (auto &v : cand) v.resize(row);
  for (int y = 0; y < h; ++y) {
    const uint8_t *cur = img + (size_t)y * row;
    const uint8_t *up = y ? cur - row : nullptr;
    long best = -1;
    int bf = 0;
    for (int f = 0; f < 5; ++f) {
      uint8_t *d = cand[f].data();
      long sum = 0;
      for (size_t i = 0; i < row; ++i) {
        const int a = i >= (size_t)c ? cur[i - c] : 0;
        const int b = up ? up[i] : 0;
        const int cc = (up && i >= (size_t)c) ? up[i - c] : 0;
        int v = cur[i];
        switch (f) {
          case 1: v -= a; break;
          case 2: v -= b; break;
          case 3: v -= (a + b) >> 1; break;
          case 4: v -= paeth(a, b, cc); break;
          default: break;
        }
        d[i] = (uint8_t)v;
        sum += d[i] < 128 ? d[i] : 256 - d[i];
      }
      if (best < 0 || sum < best) { best = sum; bf = f; }
    }
    uint8_t *o = out.data() + (size_t)y * (row + 1);
    o[0] = (uint8_t)bf;
    memcpy(o + 1, cand[bf].data(), row);
  }
}

int encode(int h, int w, int c, const uint8_t *img, int level, std::vector<uint8_t> &png) {
  std::vector<uint8_t> raw;
  filter_rows(h, w, c, img, raw);
  uLongf zlen = compressBound((uLong)raw.size());
  std::vector<uint8_t> z(zlen);
  if (compress2(z.data(), &zlen, raw.data(), (uLong)raw.size(), level) != Z_OK) return RR_ELAUNCH;
  static const uint8_t sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
  png.assign(sig, sig + 8);
  uint8_t ihdr[13];
  const uint32_t W = (uint32_t)w, H = (uint32_t)h;
  ihdr[0] = W >> 24; ihdr[1] = (W >> 16) & 255; ihdr[2] = (W >> 8) & 255; ihdr[3] = W & 255;
  ihdr[4] = H >> 24; ihdr[5] = (H >> 16) & 255; ihdr[6] = (H >> 8) & 255; ihdr[7] = H & 255;
  ihdr[8] = 8;                       // bit depth
  ihdr[9] = c == 3 ? 2 : 0;          // truecolour / greyscale
  ihdr[10] = ihdr[11] = ihdr[12] = 0;
  chunk(png, "IHDR", ihdr, 13);
  chunk(png, "IDAT", z.data(), zlen);
  chunk(png, "IEND", nullptr, 0);
  return RR_OK;
}

}  // namespace

extern "C" long long rr_png_encode(int h, int w, int c, const uint8_t *hwc, int level, uint8_t *out,
                                   long long cap) {
  if (!hwc || h <= 0 || w <= 0 || (c != 1 && c != 3) || level < 0 || level > 9) return RR_EINVAL;
  std::vector<uint8_t> png;
  if (const int rc = encode(h, w, c, hwc, level, png)) return rc;
  if (out && (long long)png.size() <= cap) memcpy(out, png.data(), png.size());
  return (long long)png.size();
}

extern "C" int rr_png_write_batch(int n, int h, int w, int c, const uint8_t *hwc,
                                  const char *const *paths, int level, int threads) {
  if (n < 0 || !paths || (n > 0 && !hwc) || h <= 0 || w <= 0 || (c != 1 && c != 3) || level < 0 ||
      level > 9)
    return RR_EINVAL;
  for (int i = 0; i < n; ++i)
    if (!paths[i]) return RR_EINVAL;
  int T = threads > 0 ? threads : (int)std::thread::hardware_concurrency();
  T = std::max(1, std::min(T, n));
  std::atomic<int> next(0), status(RR_OK);
  const size_t img = (size_t)h * w * c;
  auto work = [&]() {
    std::vector<uint8_t> png;
    for (int i = next++; i < n; i = next++) {
      if (encode(h, w, c, hwc + img * i, level, png) != RR_OK) { status = RR_ELAUNCH; continue; }
      FILE *f = fopen(paths[i], "wb");
      if (!f || fwrite(png.data(), 1, png.size(), f) != png.size()) status = RR_EINVAL;
      if (f) fclose(f);
    }
  };
  std::vector<std::thread> pool;
  for (int t = 1; t < T; ++t) pool.emplace_back(work);
  work();
  for (auto &t : pool) t.join();
  return status.load();
}
