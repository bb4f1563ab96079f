// ccj_tuning.h — tuning overrides, compiled into the TUNING build only (make tuning ->
// libccj_tuning.so, -DCCJ_TUNING; tools/ and bench.py --lib tuning use it for A/B sweeps).
// The product library (libccj.so) never reads the environment: every knob below is a compile-time
// default there, and the timing-only ablations (CCJ_ABLATE) compile to nothing.
#pragma once

#ifdef CCJ_TUNING
#include <cstdlib>
// Value of the tuning variable `name`, or nullptr.
inline const char *ccj_tune_env(const char *name) {
  const char *e = std::getenv(name);
  return e && *e ? e : nullptr;
}
inline int ccj_tune_int(const char *name, int def) {
  const char *e = ccj_tune_env(name);
  return e ? std::atoi(e) : def;
}
// Timing-only ablation bit `bit` of ProbeParams::ablate / the split's ablate word.
#define CCJ_ABLATED(word, bit) (((word) & (bit)) != 0u)
// In-kernel phase stamp (scalar time counter read; the wait keeps lgkmcnt accounting exact).
#define CCJ_STAMP(t)                                                                  \
  do {                                                                                \
    __builtin_amdgcn_sched_barrier(0);                                                \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");       \
    __builtin_amdgcn_sched_barrier(0);                                                \
  } while (0)
#else
inline const char *ccj_tune_env(const char *) { return nullptr; }
inline int ccj_tune_int(const char *, int def) { return def; }
#define CCJ_ABLATED(word, bit) (false)
#define CCJ_STAMP(t) \
  do {               \
    (t) = 0;         \
  } while (0)
#endif
