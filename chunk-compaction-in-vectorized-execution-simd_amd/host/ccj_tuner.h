// ccj_tuner.h — the compaction-threshold tuner: a UCB-tuned multi-armed bandit per join.
//
// Restates negative_feedback.hpp:20-260 (MultiArmedBandit + CompactTuner) on the host; its use
// follows main.cpp:131-167 under flag_dynamic_compact: before join l runs, SelectArm(l) picks a
// compaction threshold, and afterwards UpdateArm(l, threshold, reward) feeds back a reward that
// grows with speed.  The reference's DynamicCompactor that would consume the threshold is only
// named (setting.h:23-25); here the threshold drives the device compactor
// (ccj_pipeline_set_thresholds / ccj_compact_args.threshold): Next results of at least that many
// rows pass through, smaller ones are compacted.  An arm value a maps to threshold max(a, 1), so
// arm 0 compacts nothing and arms >= kBlockSize are the full NaiveCompactor.  The GPU decides per
// pipeline run (every join of all input chunks at once), not per chunk: one run is the unit a
// device pipeline can time without stalling it.
//
// Algorithm (negative_feedback.hpp):
//   - warm-up: every arm is pulled kStartSampling times, round robin (:35-45);
//   - then arm = argmax(est_reward + UCB-tuned bonus) (:47-61, :120-124), with
//     bonus = sqrt(ln(n) / (n_arm + eps) * min(1/4, var_arm + sqrt(2 ln(n) / (n_arm + eps))));
//   - update: exponential moving average with weight min(n_arm, 15) / (min(n_arm, 15) + 1) on
//     the old estimate, for the reward and its square (:84-90);
//   - restart: every kHeart selections, if the updated arm's estimate moved beyond [1/2, 2] of
//     its value at the previous check, estimates and counts are reset and warm-up restarts
//     (:66-82) — the workload changed.
#pragma once

#include <algorithm>
#include <cmath>
#include <cstddef>
#include <cstdint>
#include <vector>

namespace simd_compaction_amd {

class MultiArmedBandit {
 public:
  explicit MultiArmedBandit(size_t n_arms)
      : arms_(n_arms), est_(n_arms, 0.0), est_sq_(n_arms, 0.0), n_select_(n_arms, 0), n_update_(n_arms, 0) {}

  size_t SelectArm() {
    size_t arm = 0;
    if (warmup_ < arms_ * kStartSampling) {
      arm = warmup_ % arms_;
      ++warmup_;
    } else {
      double best = -1.0;
      for (size_t i = 0; i < arms_; ++i) {
        const double v = est_[i] + Bonus(i);
        if (v > best) {
          best = v;
          arm = i;
        }
      }
    }
    ++selections_;
    ++n_select_[arm];
    return arm;
  }

  void UpdateArm(size_t arm, double reward) {
    if (arm >= arms_) return;
    if (selections_ % kHeart == 0 && warmup_ >= arms_ * kStartSampling) {
      if (checkpoint_.empty()) checkpoint_ = est_;
      const bool shifted = est_[arm] > checkpoint_[arm] * 2 || est_[arm] < checkpoint_[arm] / 2;
      checkpoint_ = est_;
      if (shifted) {
        ++restarts_;
        warmup_ = 0;
        std::fill(est_.begin(), est_.end(), 0.0);
        std::fill(est_sq_.begin(), est_sq_.end(), 0.0);
        std::fill(n_update_.begin(), n_update_.end(), 0);
        updates_ = 0;
      }
    }
    const double k = (double)std::min<size_t>(n_update_[arm], 15);
    const double keep = k / (k + 1.0);
    est_[arm] = est_[arm] * keep + reward * (1.0 - keep);
    est_sq_[arm] = est_sq_[arm] * keep + reward * reward * (1.0 - keep);
    ++updates_;
    ++n_update_[arm];
  }

  size_t arms() const { return arms_; }
  double Estimate(size_t arm) const { return est_[arm]; }
  size_t Selections(size_t arm) const { return n_select_[arm]; }
  size_t Restarts() const { return restarts_; }

  static constexpr size_t kStartSampling = 4;
  static constexpr size_t kHeart = 256;

 private:
  double Bonus(size_t arm) const {
    const double n = (double)std::max<size_t>(updates_, 1);
    const double na = (double)n_update_[arm] + kEpsilon;
    const double var = est_sq_[arm] - est_[arm] * est_[arm] + std::sqrt(2.0 * std::log(n) / na);
    return std::sqrt(std::log(n) / na * std::min(0.25, var));
  }

  static constexpr double kEpsilon = 0.1;
  size_t arms_;
  std::vector<double> est_, est_sq_, checkpoint_;
  std::vector<size_t> n_select_, n_update_;
  size_t selections_ = 0, updates_ = 0, warmup_ = 0, restarts_ = 0;
};

// One bandit per compactor (join), arms = candidate thresholds (negative_feedback.hpp:160-166:
// {0, 32, ..., 1024} rows).  Arm values are mapped to thresholds for this chunk size and
// duplicates dropped (with kBlockSize 256, every arm >= 256 is the same NaiveCompactor).
class CompactTuner {
 public:
  CompactTuner(size_t n_joins, uint32_t chunk, const std::vector<uint32_t> &arms = {0, 32, 64, 128, 256, 384, 512, 768, 1024}) {
    for (uint32_t a : arms) {
      const uint32_t t = a == 0 ? 1u : std::min(a, chunk);
      if (std::find(thr_.begin(), thr_.end(), t) == thr_.end()) thr_.push_back(t);
    }
    for (size_t l = 0; l < n_joins; ++l) bandits_.emplace_back(thr_.size());
  }

  // Arm index chosen for join l, and its threshold (ccj_pipeline_set_thresholds).
  size_t SelectArm(size_t l) { return bandits_[l].SelectArm(); }
  void UpdateArm(size_t l, size_t arm, double reward) { bandits_[l].UpdateArm(arm, reward); }
  uint32_t Threshold(size_t arm) const { return thr_[arm]; }
  const std::vector<uint32_t> &thresholds() const { return thr_; }
  const MultiArmedBandit &bandit(size_t l) const { return bandits_[l]; }

 private:
  std::vector<uint32_t> thr_;
  std::vector<MultiArmedBandit> bandits_;
};

}  // namespace simd_compaction_amd
