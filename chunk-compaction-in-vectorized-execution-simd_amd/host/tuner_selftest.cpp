// tuner_selftest.cpp — CPU check of ccj_tuner.h (tests/test_tuner_cpu.py builds and runs it).
// Synthetic rewards: arm a pays mean(a) + uniform noise.  Prints one line per scenario:
//   <scenario> <selections of each arm...> restarts <n>
#include <cstdio>
#include <random>

#include "ccj_tuner.h"

using simd_compaction_amd::CompactTuner;

static void Run(const char *name, size_t rounds, size_t shift_at, unsigned seed) {
  CompactTuner t(1, 256);  // thresholds {1, 32, 64, 128, 256}
  std::mt19937 g(seed);
  std::uniform_real_distribution<double> noise(-0.05, 0.05);
  const size_t n = t.thresholds().size();
  std::vector<size_t> late(n, 0);
  for (size_t r = 0; r < rounds; ++r) {
    const size_t a = t.SelectArm(0);
    // before the shift threshold 64 is best; after it the workload is 4x faster overall (the
    // detector's trigger) and 256 is best by far
    const double mean = r < shift_at ? (a == 2 ? 1.0 : 0.5 + 0.05 * (double)a) : (a == 4 ? 8.0 : 4.0 * (0.5 + 0.05 * (double)a));
    t.UpdateArm(0, a, mean + noise(g));
    if (r + 300 >= rounds) ++late[a];
  }
  printf("%s", name);
  for (size_t a = 0; a < n; ++a) printf(" %zu", late[a]);
  printf(" restarts %zu\n", t.bandit(0).Restarts());
}

int main() {
  Run("stationary", 1000, 1u << 30, 1);
  Run("shift", 1600, 700, 2);
  return 0;
}
