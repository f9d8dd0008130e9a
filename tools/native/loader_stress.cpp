// Host-side stress test of the native data loader (csrc/runtime/loader.cpp) for the sanitizer
// builds: many short-lived loaders with more worker threads than images, shuffled
// and repeating epochs, augmentation on — the conditions of the two races fixed in round 1
// (concurrent cache fill, epoch-permutation cache eviction).  Usage: loader_stress <png dir> [iters]
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "loader.h"

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: %s <dir with i0.png i1.png m0.png m1.png> [iters]\n", argv[0]);
    return 2;
  }
  const std::string d = argv[1];
  const int iters = argc > 2 ? std::atoi(argv[2]) : 50;
  const std::vector<std::string> im = {d + "/i0.png", d + "/i1.png"}, mk = {d + "/m0.png", d + "/m1.png"};
  long batches = 0;
  for (int it = 0; it < iters; ++it) {
    tdl_rt::AugConfig aug;  // every knob on: crop and brightness paths under the sanitizers too
    aug.crop_probability = 0.5;
    aug.brightness_range = 0.2;
    tdl_rt::BatchLoader L(im, mk, 4, true, true, true, (uint64_t)it, 8, 8, 8, 0, aug);
    tdl_rt::Batch b;
    for (int k = 0; k < 3; ++k) batches += L.next(b) ? 1 : 0;
    tdl_rt::BatchLoader E(im, mk, 3, false, false, false, 0, 4, 2, 8, 1);  // eval + TTA
    while (E.next(b)) ++batches;
  }
  std::printf("ok %ld batches\n", batches);
  return 0;
}
