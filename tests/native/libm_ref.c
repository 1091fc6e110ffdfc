/* Test helper: evaluates the host glibc libm functions the reference calls,
 * exactly as the reference's expressions do (ddf.cpp:96-107, ddf_detail.h:82,
 * glm/ext/matrix_transform.inl:21-22), so tests can compare ipt_math.h to
 * them bit-for-bit. Built by tests/conftest.py with gcc -O2 -ffp-contract=off. */
#define _GNU_SOURCE
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>

typedef struct { int fn; const float* in; float* out; long lo, hi; } job_t;

static float eval1(int fn, float x) {
    float s, c;
    switch (fn) {
        case 0: return acosf(x);
        case 1: return sinf(x);
        case 2: return cosf(x);
        case 3: return (float)acos((double)x);
        case 4: sincosf(x, &s, &c); return s;
        case 5: sincosf(x, &s, &c); return c;
        case 6: return sqrtf(x);
        case 7: return (float)((double)x / M_PI);
        case 8: return (float)(2 * M_PI * (double)x);
        case 13: return sqrtf(x);
        case 14:
        case 15: {
            /* RotateDdf: cosinus = dot((0,0,1), to) for to = (0.6, 0.8, x),
             * a = (float)acos((double)cosinus) (ddf_detail.h:82), glm::rotate's
             * cos(a), sin(a) (matrix_transform.inl:21-22) */
            const float cosinus = (0.0f * 0.6f + 0.0f * 0.8f) + 1.0f * x;
            const float a = (float)acos((double)cosinus);
            return fn == 14 ? sinf(a) : cosf(a);
        }
    }
    return 0.0f;
}
static void* run(void* a) {
    job_t* j = (job_t*)a;
    for (long i = j->lo; i < j->hi; ++i) j->out[i] = eval1(j->fn, j->in[i]);
    return 0;
}
void libm_eval(int fn, const float* in, float* out, long n, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 64) nthreads = 64;
    pthread_t th[64];
    job_t jobs[64];
    for (int t = 0; t < nthreads; ++t) {
        jobs[t].fn = fn; jobs[t].in = in; jobs[t].out = out;
        jobs[t].lo = n * t / nthreads; jobs[t].hi = n * (t + 1) / nthreads;
        pthread_create(&th[t], 0, run, &jobs[t]);
    }
    for (int t = 0; t < nthreads; ++t) pthread_join(th[t], 0);
}
