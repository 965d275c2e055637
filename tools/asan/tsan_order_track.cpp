// ThreadSanitizer harness (tools/asan/Makefile `tsan`): rpt_order_and_track -- cluster order on a
// producer thread ahead of the tracker -- over synthetic stacks of 300-1000 frames.
#include <cstdio>
#include <random>
#include <vector>
#include "rpt.h"
int main() {
  std::mt19937 rng(7);
  for (int rep = 0; rep < 20; ++rep) {
    const int F = 300 + rep * 37;
    std::vector<int32_t> fr, lab;
    std::vector<int64_t> first, noise(F, -1);
    std::vector<float> cx, cy;
    for (int f = 0; f < F; ++f) {
      const int k = (int)(rng() % 40);
      for (int i = 0; i < k; ++i) {
        fr.push_back(f);
        lab.push_back((int32_t)(f * 64 + i));
        first.push_back((int64_t)(rng() % 1000000));
        cx.push_back((float)(rng() % 4000) / 10.f - 200.f);
        cy.push_back((float)(rng() % 4000) / 10.f - 200.f);
      }
      if (rng() % 2) noise[f] = (int64_t)(rng() % 1000000);
    }
    std::vector<int64_t> built;
    for (int f = 0; f < F; ++f) if (rng() % 10) built.push_back(f);
    std::vector<int64_t> fo(F + 1), order(fr.size() + 1);
    rpt_tracker* t = rpt_tracker_new(nullptr);
    const int32_t r = rpt_order_and_track(F, (int64_t)fr.size(), fr.data(), lab.data(), first.data(),
                                          noise.data(), cx.data(), cy.data(), (int32_t)built.size(),
                                          built.data(), nullptr, t, fo.data(), order.data());
    if (r != 0) { std::printf("error %d\n", r); return 1; }
    std::printf("rep %d: %d objects\n", rep, rpt_tracker_num_objects(t));
    rpt_tracker_free(t);
  }
  return 0;
}
