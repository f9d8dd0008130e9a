// Native host-side data pipeline (replaces the reference's tf.data C++ runtime + DecodeJpeg/PNG +
// ImageProjectiveTransform on the CPU, preprocessing.py:91-246, model.py:285-324).
//
//  * PNG decoder (zlib inflate + the five scanline filters; 8/16-bit gray, gray+alpha, RGB, RGBA,
//    palette) → grayscale float in [0,1]; decoded images are cached in memory (the TGS set is
//    4000 × 101² ≈ 40 MB);
//  * reference augmentation per sample: (x−MEAN)/STD → REFLECT pad 40 → random transpose →
//    H-flip / V-flip projective matrices (the reference's [-1,0,width,...] form) → rotation ±10°
//    about the centre (angles_to_projective_transforms) → translation ±20% drawn PER SAMPLE
//    (defect D13 fixed; the reference drew it once at graph construction) → optional random crop
//    (crop_probability, crop_min/max_percent) and brightness delta → composed transform
//    (M = T1·T2·…, output→input mapping as tf.contrib.image.transform) → bilinear (image) /
//    nearest (mask) sampling with zero fill → central crop → 3×3 Laplacian channel (SAME, zero pad);
//  * a worker-thread pool assembles whole batches ahead of the consumer (prefetch queue), shuffling
//    with a per-epoch permutation; output layout is the kernels' NHWC bf16 with channels padded
//    to 8 (ch0 image, ch1 Laplacian), masks fp32 [B,H,W,1].
#include "loader.h"

#include <zlib.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <fstream>
#include <stdexcept>

namespace tdl_rt {

// ------------------------------------------------------------------------------------------ PNG
static uint32_t be32(const uint8_t* p) {
  return (uint32_t(p[0]) << 24) | (uint32_t(p[1]) << 16) | (uint32_t(p[2]) << 8) | p[3];
}

static uint8_t paeth(int a, int b, int c) {
  int p = a + b - c, pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - c);
  if (pa <= pb && pa <= pc) return (uint8_t)a;
  if (pb <= pc) return (uint8_t)b;
  return (uint8_t)c;
}

GrayImage decode_png_gray(const std::vector<uint8_t>& f) {
  static const uint8_t sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
  if (f.size() < 8 || memcmp(f.data(), sig, 8) != 0) throw std::runtime_error("not a PNG file");
  size_t off = 8;
  uint32_t w = 0, h = 0;
  int depth = 0, ctype = 0, interlace = 0;
  std::vector<uint8_t> idat, plte;
  while (off + 12 <= f.size()) {
    const uint32_t len = be32(&f[off]);
    const char* type = (const char*)&f[off + 4];
    const uint8_t* data = &f[off + 8];
    if (off + 12 + len > f.size()) throw std::runtime_error("truncated PNG chunk");
    if (!memcmp(type, "IHDR", 4)) {
      w = be32(data);
      h = be32(data + 4);
      depth = data[8];
      ctype = data[9];
      interlace = data[12];
    } else if (!memcmp(type, "PLTE", 4)) {
      plte.assign(data, data + len);
    } else if (!memcmp(type, "IDAT", 4)) {
      idat.insert(idat.end(), data, data + len);
    } else if (!memcmp(type, "IEND", 4)) {
      break;
    }
    off += 12 + len;
  }
  if (interlace) throw std::runtime_error("interlaced PNG not supported");
  if (depth != 8 && depth != 16) throw std::runtime_error("PNG bit depth must be 8 or 16");
  int ch;
  switch (ctype) {
    case 0: ch = 1; break;
    case 2: ch = 3; break;
    case 3: ch = 1; break;
    case 4: ch = 2; break;
    case 6: ch = 4; break;
    default: throw std::runtime_error("unsupported PNG color type");
  }
  const int bpp = ch * depth / 8;
  const size_t stride = (size_t)w * bpp;
  std::vector<uint8_t> raw((stride + 1) * h);
  z_stream zs{};
  if (inflateInit(&zs) != Z_OK) throw std::runtime_error("inflateInit failed");
  zs.next_in = idat.data();
  zs.avail_in = (uInt)idat.size();
  zs.next_out = raw.data();
  zs.avail_out = (uInt)raw.size();
  const int zr = inflate(&zs, Z_FINISH);
  inflateEnd(&zs);
  if (zr != Z_STREAM_END && zs.avail_out != 0) throw std::runtime_error("PNG inflate failed");
  std::vector<uint8_t> px(stride * h);
  for (uint32_t y = 0; y < h; ++y) {
    const uint8_t ft = raw[y * (stride + 1)];
    const uint8_t* src = &raw[y * (stride + 1) + 1];
    uint8_t* dst = &px[y * stride];
    const uint8_t* prev = y ? &px[(y - 1) * stride] : nullptr;
    for (size_t i = 0; i < stride; ++i) {
      const int a = i >= (size_t)bpp ? dst[i - bpp] : 0;
      const int b = prev ? prev[i] : 0;
      const int c = (prev && i >= (size_t)bpp) ? prev[i - bpp] : 0;
      int v = src[i];
      switch (ft) {
        case 0: break;
        case 1: v += a; break;
        case 2: v += b; break;
        case 3: v += (a + b) / 2; break;
        case 4: v += paeth(a, b, c); break;
        default: throw std::runtime_error("bad PNG filter");
      }
      dst[i] = (uint8_t)v;
    }
  }
  GrayImage img;
  img.h = (int)h;
  img.w = (int)w;
  img.px.resize((size_t)w * h);
  const float maxv = depth == 16 ? 65535.f : 255.f;
  auto sample = [&](const uint8_t* p, int k) -> float {
    return depth == 16 ? float((p[2 * k] << 8) | p[2 * k + 1]) : float(p[k]);
  };
  for (size_t i = 0; i < (size_t)w * h; ++i) {
    const uint8_t* p = &px[i * bpp];
    float g;
    if (ctype == 0 || ctype == 4) {
      g = sample(p, 0);
    } else if (ctype == 3) {
      const int idx = p[0];
      if ((size_t)idx * 3 + 2 >= plte.size()) throw std::runtime_error("bad palette index");
      g = 0.2989f * plte[idx * 3] + 0.5870f * plte[idx * 3 + 1] + 0.1140f * plte[idx * 3 + 2];
    } else {
      g = 0.2989f * sample(p, 0) + 0.5870f * sample(p, 1) + 0.1140f * sample(p, 2);
    }
    img.px[i] = g / maxv;
  }
  return img;
}

GrayImage load_png_gray(const std::string& path) {
  std::ifstream in(path, std::ios::binary);
  if (!in) throw std::runtime_error("cannot open " + path);
  std::vector<uint8_t> buf((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
  return decode_png_gray(buf);
}

// ------------------------------------------------------------------------------ image utilities
static inline int reflect_idx(int i, int n) {  // tf.pad REFLECT (edge not repeated)
  if (n == 1) return 0;
  while (i < 0 || i >= n) {
    if (i < 0) i = -i;
    if (i >= n) i = 2 * (n - 1) - i;
  }
  return i;
}

// 3×3 matrices for the projective chain (row-major a0 a1 a2 / b0 b1 b2 / c0 c1 1)
struct Mat3 {
  double m[9];
};
static Mat3 mul(const Mat3& A, const Mat3& B) {
  Mat3 C{};
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      double s = 0;
      for (int k = 0; k < 3; ++k) s += A.m[i * 3 + k] * B.m[k * 3 + j];
      C.m[i * 3 + j] = s;
    }
  return C;
}
static Mat3 from_flat(const double t[8]) { return Mat3{{t[0], t[1], t[2], t[3], t[4], t[5], t[6], t[7], 1.0}}; }

void make_transform(const AugParams& p, int H, int W, double out[8]) {
  const double width = W, height = H;
  const double ident[8] = {1, 0, 0, 0, 1, 0, 0, 0};
  const double hflip[8] = {-1, 0, width, 0, 1, 0, 0, 0};
  const double vflip[8] = {1, 0, 0, 0, -1, height, 0, 0};
  Mat3 M = from_flat(p.hflip ? hflip : ident);
  M = mul(M, from_flat(p.vflip ? vflip : ident));
  const double c = std::cos(p.angle), s = std::sin(p.angle);
  const double xo = ((width - 1) - (c * (width - 1) - s * (height - 1))) / 2.0;
  const double yo = ((height - 1) - (s * (width - 1) + c * (height - 1))) / 2.0;
  const double rot[8] = {c, -s, xo, s, c, yo, 0, 0};
  M = mul(M, from_flat(rot));
  const double tr[8] = {1, 0, p.tx, 0, 1, p.ty, 0, 0};
  M = mul(M, from_flat(tr));
  if (p.crop) {
    // the reference's crop transform, offsets as written there (top in the x row, left in the
    // y row: preprocessing.py:219-221)
    const double cr[8] = {p.crop_pct, 0, p.crop_top, 0, p.crop_pct, p.crop_left, 0, 0};
    M = mul(M, from_flat(cr));
  }
  for (int i = 0; i < 8; ++i) out[i] = M.m[i] / M.m[8];
}

template <class RNG>
AugParams draw_aug(const AugConfig& cfg, int H, int W, RNG& rng) {
  std::uniform_real_distribution<double> U(0.0, 1.0);
  AugParams p;
  p.transpose = U(rng) > 0.5;
  if (cfg.brightness_range > 0) p.brightness = (2 * U(rng) - 1) * cfg.brightness_range;
  if (cfg.horizontal_flip) p.hflip = U(rng) < 0.5;
  if (cfg.vertical_flip) p.vflip = U(rng) < 0.5;
  const double ar = cfg.rotate_range / 180.0 * M_PI;
  p.angle = -ar + 2 * ar * U(rng);
  // both shifts scale with the height in the reference (preprocessing.py:196-203); drawn per
  // sample here (defect D13 fixed)
  p.tx = cfg.width_shift_range ? (2 * U(rng) - 1) * cfg.width_shift_range * H : 0.0;
  p.ty = cfg.height_shift_range ? (2 * U(rng) - 1) * cfg.height_shift_range * H : 0.0;
  if (cfg.crop_probability > 0) {
    p.crop_pct = cfg.crop_min_percent + (cfg.crop_max_percent - cfg.crop_min_percent) * U(rng);
    p.crop_left = U(rng) * W * (1 - p.crop_pct);
    p.crop_top = U(rng) * H * (1 - p.crop_pct);
    p.crop = U(rng) < cfg.crop_probability;
  }
  return p;
}
template AugParams draw_aug<std::mt19937_64>(const AugConfig&, int, int, std::mt19937_64&);

// tf.contrib.image.transform: output (x, y) samples input at (a0x+a1y+a2, b0x+b1y+b2)/(c0x+c1y+1)
void projective_warp(const float* in, int H, int W, const double t[8], bool nearest, float* out) {
  for (int y = 0; y < H; ++y)
    for (int x = 0; x < W; ++x) {
      const double k = t[6] * x + t[7] * y + 1.0;
      const double ix = (t[0] * x + t[1] * y + t[2]) / k;
      const double iy = (t[3] * x + t[4] * y + t[5]) / k;
      float v = 0.f;
      if (nearest) {
        const long rx = std::lround(ix), ry = std::lround(iy);
        if (rx >= 0 && rx < W && ry >= 0 && ry < H) v = in[ry * W + rx];
      } else {
        const double fx = std::floor(ix), fy = std::floor(iy);
        const double ax = ix - fx, ay = iy - fy;
        const long x0 = (long)fx, y0 = (long)fy;
        auto at = [&](long yy, long xx) -> double {
          return (xx >= 0 && xx < W && yy >= 0 && yy < H) ? in[yy * W + xx] : 0.0;
        };
        v = (float)((1 - ay) * ((1 - ax) * at(y0, x0) + ax * at(y0, x0 + 1)) +
                    ay * ((1 - ax) * at(y0 + 1, x0) + ax * at(y0 + 1, x0 + 1)));
      }
      out[y * W + x] = v;
    }
}

void laplace(const float* in, int H, int W, float* out) {
  static const float k[3][3] = {{0.5f, 1.f, 0.5f}, {1.f, -6.f, 1.f}, {0.5f, 1.f, 0.5f}};
  for (int y = 0; y < H; ++y)
    for (int x = 0; x < W; ++x) {
      float s = 0.f;
      for (int dy = -1; dy <= 1; ++dy)
        for (int dx = -1; dx <= 1; ++dx) {
          const int yy = y + dy, xx = x + dx;
          if (yy >= 0 && yy < H && xx >= 0 && xx < W) s += k[dy + 1][dx + 1] * in[yy * W + xx];
        }
      out[y * W + x] = s;
    }
}

void augment_sample(const GrayImage& img, const GrayImage* mask, const AugParams& p, int pad,
                    float* out_img, float* out_mask) {
  const int H = img.h, W = img.w;
  const int PH = H + 2 * pad, PW = W + 2 * pad;
  std::vector<float> pi((size_t)PH * PW), pm(mask ? (size_t)PH * PW : 0);
  for (int y = 0; y < PH; ++y)
    for (int x = 0; x < PW; ++x) {
      int sy = reflect_idx(y - pad, H), sx = reflect_idx(x - pad, W);
      if (p.transpose) std::swap(sy, sx);  // transpose_image (square images)
      pi[(size_t)y * PW + x] = (img.px[(size_t)sy * W + sx] - MEAN) / STD + (float)p.brightness;
      if (mask) pm[(size_t)y * PW + x] = mask->px[(size_t)sy * W + sx];
    }
  double t[8];
  make_transform(p, PH, PW, t);
  std::vector<float> wi((size_t)PH * PW), wm(mask ? (size_t)PH * PW : 0);
  projective_warp(pi.data(), PH, PW, t, false, wi.data());
  if (mask) projective_warp(pm.data(), PH, PW, t, true, wm.data());
  // central crop back to H×W
  const int oy = (PH - H) / 2, ox = (PW - W) / 2;
  for (int y = 0; y < H; ++y)
    for (int x = 0; x < W; ++x) {
      out_img[(size_t)y * W + x] = wi[(size_t)(y + oy) * PW + x + ox];
      if (mask) out_mask[(size_t)y * W + x] = wm[(size_t)(y + oy) * PW + x + ox];
    }
}

void single_transformation(const float* in, int H, int W, int kind, float* out) {
  // kind: 0 none, 1 vertical (flip_up_down), 2 horizontal (flip_left_right), 3 transpose
  for (int y = 0; y < H; ++y)
    for (int x = 0; x < W; ++x) {
      int sy = y, sx = x;
      if (kind == 1) sy = H - 1 - y;
      if (kind == 2) sx = W - 1 - x;
      if (kind == 3) std::swap(sy, sx);
      out[(size_t)y * W + x] = in[(size_t)sy * W + sx];
    }
}

static inline uint16_t f2bf(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return 0x7fc0;
  u += 0x7fff + ((u >> 16) & 1);
  return (uint16_t)(u >> 16);
}

// --------------------------------------------------------------------------------------- loader
BatchLoader::BatchLoader(const std::vector<std::string>& images,
                         const std::vector<std::string>& masks, int batch, bool augment,
                         bool shuffle, bool repeat, uint64_t seed, int threads, int prefetch,
                         int channels, int transformation, const AugConfig& aug, bool fp32)
    : images_(images), masks_(masks), batch_(batch), augment_(augment), shuffle_(shuffle),
      repeat_(repeat), seed_(seed), channels_(channels), transformation_(transformation),
      aug_(aug), fp32_(fp32) {
  if (aug_.crop_probability < 0 || aug_.crop_probability > 1 || aug_.brightness_range < 0 ||
      aug_.crop_min_percent <= 0 || aug_.crop_max_percent < aug_.crop_min_percent)
    throw std::runtime_error("invalid augmentation parameters");
  if (!masks_.empty() && masks_.size() != images_.size())
    throw std::runtime_error("images and masks differ in length");
  if (images_.empty()) throw std::runtime_error("empty dataset");
  if (channels_ < 2) throw std::runtime_error("channels must be >= 2 (image + Laplacian)");
  cache_img_.resize(images_.size());
  cache_mask_.resize(masks_.size());
  cached_.assign(images_.size(), 0);
  // shape from the first image
  GrayImage first = load_png_gray(images_[0]);
  H_ = first.h;
  W_ = first.w;
  prefetch_ = std::max(1, prefetch);
  const int nthreads = std::max(1, threads);
  n_batches_ = repeat_ ? -1 : (long)((images_.size() + batch_ - 1) / batch_);
  for (int i = 0; i < nthreads; ++i) workers_.emplace_back([this] { work(); });
}

BatchLoader::~BatchLoader() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    stop_ = true;
  }
  cv_work_.notify_all();
  cv_ready_.notify_all();
  for (auto& t : workers_) t.join();
}

std::vector<int64_t> BatchLoader::indices_for(long b) {
  // epoch-wise permutation (deterministic in seed and epoch)
  const long n = (long)images_.size();
  std::vector<int64_t> out(batch_);
  for (int i = 0; i < batch_; ++i) {
    const long g = b * batch_ + i;
    const long epoch = g / n, pos = g % n;
    if (!repeat_ && epoch > 0) {
      out[i] = -1;
      continue;
    }
    if (!shuffle_) {
      out[i] = pos;
      continue;
    }
    {
      std::lock_guard<std::mutex> lk(perm_mu_);
      auto it = perms_.find(epoch);
      if (it == perms_.end()) {
        std::vector<int64_t> p(n);
        for (long j = 0; j < n; ++j) p[j] = j;
        std::mt19937_64 rng(seed_ * 1000003ull + epoch);
        std::shuffle(p.begin(), p.end(), rng);
        it = perms_.emplace(epoch, std::move(p)).first;
      }
      out[i] = it->second[pos];
      // bound the cache (a regenerated old epoch is the smallest key: never evict the entry in use)
      while (perms_.size() > 8) {
        auto victim = perms_.begin();
        if (victim == it) ++victim;
        perms_.erase(victim);
      }
    }
  }
  return out;
}

const GrayImage& BatchLoader::get(std::vector<GrayImage>& cache, const std::vector<std::string>& paths,
                                  size_t i) {
  {
    std::lock_guard<std::mutex> lk(cache_mu_);
    if (&cache == &cache_img_ ? (cached_[i] & 1) : (cached_[i] & 2)) return cache[i];
  }
  GrayImage g = load_png_gray(paths[i]);
  std::lock_guard<std::mutex> lk(cache_mu_);
  // another worker may have published this entry meanwhile and be reading it: never overwrite
  const uint8_t bit = (&cache == &cache_img_) ? 1 : 2;
  if (!(cached_[i] & bit)) {
    cache[i] = std::move(g);
    cached_[i] |= bit;
  }
  return cache[i];
}

void BatchLoader::build(long b, Batch& out) {
  const auto idx = indices_for(b);
  const int HW = H_ * W_;
  out.index = b;
  if (fp32_) {
    out.xf.assign((size_t)batch_ * HW * channels_, 0.f);
    out.x.clear();
  } else {
    out.x.assign((size_t)batch_ * HW * channels_, 0);
  }
  out.y.assign(masks_.empty() ? 0 : (size_t)batch_ * HW, 0.f);
  out.ids.assign(idx.begin(), idx.end());
  out.count = 0;
  std::vector<float> img(HW), msk(HW), lap(HW), tmp(HW);
  for (int i = 0; i < batch_; ++i) {
    if (idx[i] < 0) continue;
    out.count = i + 1;
    const GrayImage& gi = get(cache_img_, images_, idx[i]);
    const GrayImage* gm = masks_.empty() ? nullptr : &get(cache_mask_, masks_, idx[i]);
    if (augment_) {
      std::mt19937_64 rng(seed_ * 7919ull + (uint64_t)b * 104729ull + i);
      const AugParams p = draw_aug(aug_, H_ + 80, W_ + 80, rng);
      augment_sample(gi, gm, p, 40, img.data(), gm ? msk.data() : nullptr);
    } else {
      for (int k = 0; k < HW; ++k) img[k] = (gi.px[k] - MEAN) / STD;
      if (gm) std::copy(gm->px.begin(), gm->px.end(), msk.begin());
      if (transformation_) {
        single_transformation(img.data(), H_, W_, transformation_, tmp.data());
        std::swap(img, tmp);
        if (gm) {
          single_transformation(msk.data(), H_, W_, transformation_, tmp.data());
          std::swap(msk, tmp);
        }
      }
    }
    laplace(img.data(), H_, W_, lap.data());
    if (fp32_) {
      float* xo = &out.xf[(size_t)i * HW * channels_];
      for (int k = 0; k < HW; ++k) {
        xo[(size_t)k * channels_] = img[k];
        xo[(size_t)k * channels_ + 1] = lap[k];
      }
    } else {
      uint16_t* xo = &out.x[(size_t)i * HW * channels_];
      for (int k = 0; k < HW; ++k) {
        xo[(size_t)k * channels_] = f2bf(img[k]);
        xo[(size_t)k * channels_ + 1] = f2bf(lap[k]);
      }
    }
    if (gm) std::copy(msk.begin(), msk.end(), out.y.begin() + (size_t)i * HW);
  }
}

void BatchLoader::work() {
  for (;;) {
    long b;
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_work_.wait(lk, [&] {
        return stop_ || (next_to_build_ < next_to_take_ + prefetch_ &&
                         (n_batches_ < 0 || next_to_build_ < n_batches_));
      });
      if (stop_) return;
      b = next_to_build_++;
    }
    Batch bt;
    std::string err;
    try {
      build(b, bt);
    } catch (const std::exception& e) {
      err = e.what();
    }
    {
      std::lock_guard<std::mutex> lk(mu_);
      if (!err.empty()) error_ = err;
      ready_.emplace(b, std::move(bt));
    }
    cv_ready_.notify_all();
  }
}

bool BatchLoader::next(Batch& out) {
  std::unique_lock<std::mutex> lk(mu_);
  if (n_batches_ >= 0 && next_to_take_ >= n_batches_) return false;
  const long want = next_to_take_;
  cv_work_.notify_all();
  cv_ready_.wait(lk, [&] { return stop_ || !error_.empty() || ready_.count(want); });
  if (!error_.empty()) throw std::runtime_error(error_);
  if (stop_) return false;
  out = std::move(ready_[want]);
  ready_.erase(want);
  ++next_to_take_;
  lk.unlock();
  cv_work_.notify_all();
  return true;
}

}  // namespace tdl_rt
