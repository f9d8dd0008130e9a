// Native host data pipeline (see loader.cpp).
#pragma once
#include <condition_variable>
#include <cstdint>
#include <map>
#include <mutex>
#include <random>
#include <string>
#include <thread>
#include <vector>

namespace tdl_rt {

constexpr float MEAN = 0.47194585f;  // preprocessing.py:7-8
constexpr float STD = 0.16105755f;

struct GrayImage {
  int h = 0, w = 0;
  std::vector<float> px;  // [h*w] in [0,1]
};

GrayImage decode_png_gray(const std::vector<uint8_t>& file);
GrayImage load_png_gray(const std::string& path);

// one sample's draw of the reference augmentation (preprocessing.py:112-246)
struct AugParams {
  bool transpose = false, hflip = false, vflip = false;
  double angle = 0.0, tx = 0.0, ty = 0.0;
  double brightness = 0.0;                        // tf.image.random_brightness delta (image only)
  bool crop = false;                              // random-crop transform applied
  double crop_pct = 1.0, crop_left = 0.0, crop_top = 0.0;
};

// the knobs of read_and_preprocess (preprocessing.py:112-123), same names and defaults
struct AugConfig {
  bool horizontal_flip = true, vertical_flip = true;
  double rotate_range = 10.0;                     // degrees
  double crop_probability = 0.5, crop_min_percent = 0.9, crop_max_percent = 1.1;
  double height_shift_range = 0.2, width_shift_range = 0.2;
  double brightness_range = 0.0;
};

// draw one sample's parameters from `cfg` (padded image size H×W) — the reference's draw order:
// transpose, brightness, H-flip, V-flip, angle, shifts, crop
template <class RNG>
AugParams draw_aug(const AugConfig& cfg, int H, int W, RNG& rng);

void make_transform(const AugParams& p, int H, int W, double out[8]);
void projective_warp(const float* in, int H, int W, const double t[8], bool nearest, float* out);
void laplace(const float* in, int H, int W, float* out);
void augment_sample(const GrayImage& img, const GrayImage* mask, const AugParams& p, int pad,
                    float* out_img, float* out_mask);
void single_transformation(const float* in, int H, int W, int kind, float* out);

struct Batch {
  long index = -1;
  int count = 0;                 // valid samples (last batch of a non-repeating epoch may be short)
  std::vector<uint16_t> x;       // bf16 [B,H,W,C] (fp32 loaders: empty)
  std::vector<float> xf;         // fp32 [B,H,W,C] (fp32 loaders only)
  std::vector<float> y;          // fp32 [B,H,W] (empty without masks)
  std::vector<int64_t> ids;      // dataset indices (-1 = padding)
};

class BatchLoader {
 public:
  BatchLoader(const std::vector<std::string>& images, const std::vector<std::string>& masks,
              int batch, bool augment, bool shuffle, bool repeat, uint64_t seed, int threads,
              int prefetch, int channels, int transformation, const AugConfig& aug = AugConfig(),
              bool fp32 = false);
  ~BatchLoader();
  bool next(Batch& out);
  int height() const { return H_; }
  int width() const { return W_; }
  int channels() const { return channels_; }
  int batch() const { return batch_; }
  bool fp32() const { return fp32_; }
  long num_batches() const { return n_batches_; }

 private:
  void work();
  void build(long b, Batch& out);
  std::vector<int64_t> indices_for(long b);
  const GrayImage& get(std::vector<GrayImage>& cache, const std::vector<std::string>& paths,
                       size_t i);

  std::vector<std::string> images_, masks_;
  int batch_;
  bool augment_, shuffle_, repeat_;
  uint64_t seed_;
  int channels_, transformation_;
  AugConfig aug_;
  bool fp32_ = false;  // emit the image batch in fp32 (the reference's precision) instead of bf16
  int H_ = 0, W_ = 0, prefetch_ = 2;
  long n_batches_ = -1;
  std::vector<GrayImage> cache_img_, cache_mask_;
  std::vector<uint8_t> cached_;
  std::mutex cache_mu_, perm_mu_, mu_;
  std::map<long, std::vector<int64_t>> perms_;
  std::condition_variable cv_work_, cv_ready_;
  std::map<long, Batch> ready_;
  long next_to_build_ = 0, next_to_take_ = 0;
  bool stop_ = false;
  std::string error_;
  std::vector<std::thread> workers_;
};

}  // namespace tdl_rt
