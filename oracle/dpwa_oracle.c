/*
 * dpwa_oracle.c -- CPU restatement of dpwa's pairwise-averaging arithmetic.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker / the CPU
 * baseline.  The product path (dpwa_amd/libdpwa_hip.so) never links or calls it.
 *
 * Pinned by tests/test_oracle.py against tests/golden/lerp_f32.npz, which was
 * produced by running the reference adapter itself (tests/golden/make_golden.py).
 *
 * Reference semantics restated (zenghanfu/dpwa):
 *   dpwa/adapters/pytorch.py:68   param.data = factor * t + (1 - factor) * param.data
 * with torch-eager rounding: the Python float `factor` is cast to the fp32 op type
 * (a = f32(factor)); `1 - factor` is evaluated in Python double before the cast
 * (b = f32(1.0 - factor)); two separately rounded products and a rounded sum -- no
 * FMA contraction (this file must be compiled with -ffp-contract=off).
 * The bf16 form (reference has no bf16 path: pytorch.py:11-14) is the torch-eager
 * result for bf16 tensors: bf16(bf16(a*t) + bf16(b*p)), products/sum in fp32, RNE.
 */
#include <stdint.h>
#include <string.h>

#if defined(__FP_FAST_FMAF) || defined(__FAST_MATH__)
#error "dpwa_oracle.c must be built without fast-math / FMA contraction"
#endif

void dpwa_oracle_lerp_f32(float *param, const float *peer, int64_t n, double factor)
{
    const float a = (float)factor;
    const float b = (float)(1.0 - factor);
    for (int64_t i = 0; i < n; ++i) {
        float x = a * peer[i];   /* -ffp-contract=off, no -mfma: three roundings */
        float y = b * param[i];
        param[i] = x + y;
    }
}

static inline float bf16_to_f32(uint16_t h)
{
    uint32_t u = (uint32_t)h << 16;
    float f;
    memcpy(&f, &u, 4);
    return f;
}

/* c10::BFloat16 round-to-nearest-even; NaN -> canonical quiet NaN 0x7FC0. */
static inline uint16_t f32_to_bf16(float f)
{
    uint32_t u;
    memcpy(&u, &f, 4);
    if ((u & 0x7fffffffu) > 0x7f800000u)
        return 0x7FC0;
    return (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}

void dpwa_oracle_lerp_bf16(uint16_t *param, const uint16_t *peer, int64_t n, double factor)
{
    const float a = (float)factor;
    const float b = (float)(1.0 - factor);
    for (int64_t i = 0; i < n; ++i) {
        float x = bf16_to_f32(f32_to_bf16(a * bf16_to_f32(peer[i])));
        float y = bf16_to_f32(f32_to_bf16(b * bf16_to_f32(param[i])));
        param[i] = f32_to_bf16(x + y);
    }
}

/* The snapshot half of a round (dpwa/adapters/pytorch.py:49-53 copies every
 * parameter into a blob): a plain copy. */
void dpwa_oracle_publish(void *slot, const void *flat, int64_t nbytes)
{
    memcpy(slot, flat, (size_t)nbytes);
}

/* dpwa/dpwa.py:143-150 in IEEE double, separately rounded.
 * method: 0 constant(value) interpolation.py:13-15, 1 clock interpolation.py:22-24,
 *         2 loss interpolation.py:31-33.  Returns 0, or 1 on the Python
 *         ZeroDivisionError of clock+peer_clock == 0 / loss+peer_loss == 0. */
int dpwa_oracle_factor(int method, double value, double threshold, double clock,
                       double peer_clock, double loss, double peer_loss,
                       double *factor_out, double *new_clock_out)
{
    volatile double f;
    if (method == 0) {
        f = value;
    } else if (method == 1) {
        volatile double den = clock + peer_clock;
        if (den == 0.0) return 1;
        f = peer_clock / den;
    } else {
        volatile double den = loss + peer_loss;
        if (den == 0.0) return 1;
        f = loss / den;
    }
    if (loss < threshold) {
        volatile double q = loss / threshold;
        f = f * q;
    }
    volatile double t1 = f * peer_clock;
    volatile double om = 1.0 - f;
    volatile double t2 = om * clock;
    *factor_out = f;
    *new_clock_out = t1 + t2;
    return 0;
}
