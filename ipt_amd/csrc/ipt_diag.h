// ipt_diag.h — diagnostic instrumentation hooks of path_kernel. Every hook
// compiles to nothing in the product build; a diagnostic build (scripts/
// prof_phases.sh, listing builds) must say so with -DIPT_DIAGNOSTIC_BUILD, so
// that a stray -D in a product build fails to compile instead of shipping.
//
//   -DIPT_PROF=1   per phase: wave executions and active lanes in them (lane
//                  utilisation), read back with ipt_get_profile();
//   -DIPT_STAMP=1  per step segment: wave-cycles (s_memtime) since the
//                  previous stamp; read their SHARES (the stamps' waits forbid
//                  overlaps the real kernel has);
//   -DIPT_MARK=1 / -DIPT_MARK_PHASES=1  asm-listing builds: a ;@STAMP / ;@PHASE
//                  comment at each hook (per-segment instruction counts);
//   -DIPT_RAYLOG=1 every raylog_every-th finished sphere-list trace of the
//                  resumable instances (origin, direction, nearest t, hit) into
//                  a device buffer (scripts/probes/walk_split.hip, the split
//                  traversal measurement).
// None of them changes a result.
#pragma once

#ifndef IPT_PROF
#define IPT_PROF 0
#endif
#ifndef IPT_STAMP
#define IPT_STAMP 0
#endif
#ifndef IPT_MARK
#define IPT_MARK 0
#endif
#ifndef IPT_MARK_PHASES
#define IPT_MARK_PHASES 0
#endif
#ifndef IPT_RAYLOG
#define IPT_RAYLOG 0
#endif
#if (IPT_PROF || IPT_STAMP || IPT_MARK || IPT_MARK_PHASES || IPT_RAYLOG) && !defined(IPT_DIAGNOSTIC_BUILD)
#error "IPT_PROF / IPT_STAMP / IPT_MARK* / IPT_RAYLOG are diagnostic: build with -DIPT_DIAGNOSTIC_BUILD, outside ipt_amd/lib"
#endif

// IPT_RAYLOG's record: a traced ray and the walk's result (t bits, and the
// hit: sphere index >= 0, or -2 - box plane)
struct RayLogRec {
    float o[3], t;
    float d[3];
    int hit;
};

constexpr int kProfPhases = 12;
constexpr int kStamps = 12;

#define IPT_PHASE(id)                                                     \
    if (IPT_PROF) {                                                       \
        const uint64_t pm_ = __ballot(1);                                 \
        if ((int)(threadIdx.x & 63) == __ffsll((long long)pm_) - 1) {     \
            prof_w[id] += 1u;                                             \
            prof_l[id] += (uint32_t)__popcll(pm_);                        \
        }                                                                 \
    }                                                                     \
    if (IPT_MARK_PHASES) {                                                \
        __builtin_amdgcn_sched_barrier(0);                                \
        asm volatile(";@PHASE " #id);                                     \
        __builtin_amdgcn_sched_barrier(0);                                \
    }

#define IPT_STAMP_AT(id)                                                           \
    if (IPT_STAMP) {                                                               \
        unsigned long long t_;                                                     \
        __builtin_amdgcn_sched_barrier(0);                                         \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory"); \
        __builtin_amdgcn_sched_barrier(0);                                         \
        st_acc[id] += (uint32_t)(t_ - st_last);                                    \
        st_last = t_;                                                              \
    }                                                                              \
    if (IPT_MARK) {                                                                \
        __builtin_amdgcn_sched_barrier(0);                                         \
        asm volatile(";@STAMP " #id);                                              \
        __builtin_amdgcn_sched_barrier(0);                                         \
    }

// IPT_PROF: device functions with their own hooks take the arrays as extra
// parameters (nothing in other builds)
#if IPT_PROF
#define IPT_DIAG_PARAMS , uint32_t *prof_w, uint32_t *prof_l
#define IPT_DIAG_ARGS , prof_w, prof_l
#define IPT_DIAG_NULL_ARGS , nullptr, nullptr
#else
#define IPT_DIAG_NULL_ARGS
#define IPT_DIAG_PARAMS
#define IPT_DIAG_ARGS
#endif

// the hooks' per-lane state, declared at the top of the kernel
#define IPT_DIAG_STATE                                                                    \
    uint32_t prof_w[kProfPhases], prof_l[kProfPhases];                                    \
    uint32_t st_acc[kStamps];                                                             \
    unsigned long long st_last = 0;                                                       \
    if (IPT_STAMP) {                                                                      \
        for (int q = 0; q < kStamps; ++q) st_acc[q] = 0u;                                 \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(st_last)::"memory");   \
    }                                                                                     \
    if (IPT_PROF)                                                                         \
        for (int q = 0; q < kProfPhases; ++q) prof_w[q] = prof_l[q] = 0u;

// flushed at the kernel's end into words [base, base + 2*kProfPhases + kStamps)
// of the counter buffer (each wave-execution of a phase was counted by its
// lowest active lane)
#define IPT_DIAG_FLUSH(counters, base)                                                               \
    if (IPT_STAMP && lane == 0)                                                                      \
        for (int q = 0; q < kStamps; ++q)                                                            \
            atomicAdd(&(counters)[(base) + 2 * kProfPhases + q], (unsigned long long)st_acc[q]);     \
    if (IPT_PROF)                                                                                    \
        for (int q = 0; q < kProfPhases; ++q)                                                        \
            if (prof_w[q]) {                                                                         \
                atomicAdd(&(counters)[(base) + 2 * q], (unsigned long long)prof_w[q]);               \
                atomicAdd(&(counters)[(base) + 2 * q + 1], (unsigned long long)prof_l[q]);           \
            }
