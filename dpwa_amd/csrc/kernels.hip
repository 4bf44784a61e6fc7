// kernels.hip -- CDNA4 (gfx950) kernels of the pairwise-averaging hot path.
//
//  * lerp:    the averaging statement of dpwa/adapters/pytorch.py:68,
//             param = f32(f32(a*peer) + f32(b*param)), as ONE streaming pass over the flat
//             parameter buffer (the reference runs three ATen kernels and allocates three
//             temporaries per tensor).  Pure HBM streaming (0.25 flop/byte): no LDS
//             staging, no MFMA.  Shape chosen by measurement (tools/lerp_tune.hip): one
//             16-byte item per lane and an exact grid -- many short-lived one-wave
//             workgroups keep the most loads in flight per CU (tools/block_sweep.sh);
//             grid-stride loops with more items per lane or a capped grid were 5-20%
//             slower on gfx950.
//             Separate roundings are required for bit parity with the reference (an FMA
//             changes up to ~30% of results near cancellation), so contraction is
//             switched off for this whole file.
//  * fused average: the same pass with the factor of dpwa/dpwa.py:139-155 computed in
//             the kernel: every workgroup evaluates it in fp64 while its loads are in flight
//             (one-wave workgroups keep the uniform (a, b) in registers; wider ones have wave 0
//             share them through LDS); block 0
//             also writes the new clock (into the other half of a double-buffered clock,
//             so no workgroup ever reads a clock another one is writing) and dpwa_coef.
//  * factor:  the same fp64 math as a one-thread kernel for the split API.
//  * publish: update_send's snapshot (dpwa.py:111-116, pytorch.py:49-53) -- clock += 1 on
//             the device and one copy of the flat buffer into a snapshot slot behind its
//             header.
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>

#include "kernels.hpp"

#include <hip/hip_ext.h>

#ifndef DPWA_FACTOR_LDS
#define DPWA_FACTOR_LDS 0     // 1: one-wave workgroups hand the factor over through LDS too (A/B builds)
#endif
#ifndef DPWA_GROUP_FACTORS_FIRST
#define DPWA_GROUP_FACTORS_FIRST 0   // 1: group_span evaluates every entry's factor before any store (A/B builds)
#endif

namespace dpwa {

constexpr int kBlock = 256;   // 4 waves of 64

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef float float2v __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));

static inline int64_t blocks_for(int64_t items)
{
    int64_t g = (items + kBlock - 1) / kBlock;
    return g < 1 ? 1 : g;
}

// ---------------------------------------------------------------- element ops
__device__ __forceinline__ float lerp1(float a, float b, float peer, float param)
{
    float x = a * peer;     // f32(a*t)          pytorch.py:68 `factor * t`
    float y = b * param;    // f32(b*p)          pytorch.py:68 `(1 - factor) * param.data`
    return x + y;           // f32(x + y)        contraction is off for this file
}

__device__ __forceinline__ float bf_lo(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float bf_hi(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }

// Two f32 -> packed bf16, round-to-nearest-even (v_cvt_pk_bf16_f32 on gfx950).
__device__ __forceinline__ uint32_t pk_bf16(float lo, float hi)
{
    float2v v = {lo, hi};
    bf16x2v r = __builtin_convertvector(v, bf16x2v);
    return __builtin_bit_cast(uint32_t, r);
}

// bf16(bf16(a*q) + bf16(b*p)) for the two bf16 held in each 32-bit word (torch-eager form).
__device__ __forceinline__ uint32_t lerp_bf16x2(float a, float b, uint32_t q, uint32_t p)
{
    uint32_t x = pk_bf16(a * bf_lo(q), a * bf_hi(q));
    uint32_t y = pk_bf16(b * bf_lo(p), b * bf_hi(p));
    return pk_bf16(bf_lo(x) + bf_lo(y), bf_hi(x) + bf_hi(y));
}

struct OpsF32 {
    using V = f32x4;
    using S = float;
    static constexpr int PER = 4;
    __device__ static __forceinline__ V lerp(float a, float b, V q, V p)
    {
        V x = a * q;
        V y = b * p;
        return x + y;
    }
    __device__ static __forceinline__ S lerp_s(float a, float b, S q, S p) { return lerp1(a, b, q, p); }
};

struct OpsBF16 {
    using V = u32x4;
    using S = uint16_t;
    static constexpr int PER = 8;
    __device__ static __forceinline__ V lerp(float a, float b, V q, V p)
    {
        V r;
        r.x = lerp_bf16x2(a, b, q.x, p.x);
        r.y = lerp_bf16x2(a, b, q.y, p.y);
        r.z = lerp_bf16x2(a, b, q.z, p.z);
        r.w = lerp_bf16x2(a, b, q.w, p.w);
        return r;
    }
    __device__ static __forceinline__ S lerp_s(float a, float b, S q, S p)
    {
        return (S)(lerp_bf16x2(a, b, (uint32_t)q, (uint32_t)p) & 0xffffu);
    }
};

// The loss given to update_send / update_wait: a host double, or read on the device from a
// float64 or float32 scalar (a loss tensor, so the host never synchronises).
__device__ __forceinline__ double read_loss(const double *d, int32_t f32, double h)
{
    if (!d) return h;
    return f32 ? (double)*reinterpret_cast<const float *>(d) : *d;
}

// ---------------------------------------------------------------- factor math
// dpwa.py:139-155 in IEEE double with every operation separately rounded, exactly as
// CPython evaluates it.  Python raises ZeroDivisionError on x/0.0; here that is status 1,
// the clock is left unchanged and the lerp becomes a no-op.
__device__ __forceinline__ dpwa_coef factor_math(const dpwa_interp &cfg, double c, double pc, double pl, double loss)
{
    int32_t status = DPWA_STATUS_OK;
    double f = 0.0;
    if (cfg.method == DPWA_INTERP_CONSTANT) {          // interpolation.py:13-15
        f = cfg.value;
    } else if (cfg.method == DPWA_INTERP_CLOCK) {      // interpolation.py:22-24
        const double den = c + pc;
        if (den == 0.0) status = DPWA_STATUS_ZERO_DIVISION;
        else f = pc / den;
    } else {                                           // interpolation.py:31-33
        const double den = loss + pl;
        if (den == 0.0) status = DPWA_STATUS_ZERO_DIVISION;
        else f = loss / den;
    }
    if (status == DPWA_STATUS_OK && loss < cfg.divergence_threshold) {   // dpwa.py:146-147
        if (cfg.divergence_threshold == 0.0) status = DPWA_STATUS_ZERO_DIVISION;
        else f = f * (loss / cfg.divergence_threshold);
    }
    dpwa_coef out;
    out.status = status;
    out.reserved = 0;
    if (status == DPWA_STATUS_OK) {
        out.factor = f;
        out.new_clock = f * pc + (1.0 - f) * c;        // dpwa.py:150
        out.a = (float)f;                              // torch: Python float -> fp32 scalar
        out.b = (float)(1.0 - f);                      // `1 - factor` in double, then fp32
    } else {
        out.factor = 0.0;
        out.new_clock = c;
        out.a = 0.0f;
        out.b = 1.0f;
    }
    return out;
}

__device__ __forceinline__ void factor_commit(const FusedArgs &fa, const dpwa_coef &c)
{
    *fa.clock_out = c.new_clock;                       // dpwa.py:155 (unchanged on error)
    *fa.coef_out = c;
    if (fa.status_mirror && c.status != DPWA_STATUS_OK) *fa.status_mirror = c.status;   // sticky
    if (fa.next_header) {                              // the next publish's state, written ahead
        const double next = c.new_clock + 1.0;         // dpwa.py:112 of that publish
        *fa.clock_next = next;
        dpwa_header *h = fa.next_header;
        h->clock = next;
        h->loss = __builtin_nan("");
        h->version = fa.next_version;
        h->n = fa.n;
        h->dtype = fa.dtype;
    }
}

__global__ void k_factor(FusedArgs fa)
{
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    const double loss = read_loss(fa.loss_d, fa.loss_f32, fa.loss_h);
    const dpwa_coef c = factor_math(fa.cfg, *fa.clock_in, fa.hdr->clock, fa.hdr->loss, loss);
    factor_commit(fa, c);
}

hipError_t launch_factor(const FusedArgs &fa, hipStream_t s)
{
    hipLaunchKernelGGL(k_factor, dim3(1), dim3(64), 0, s, fa);
    return hipGetLastError();
}

// ---------------------------------------------------------------- lerp kernels
enum CoefMode { COEF_HOST = 0, COEF_DEV = 1, COEF_FUSED = 2 };

struct LerpArgs {
    float a, b;                  // COEF_HOST
    const dpwa_coef *coef;       // COEF_DEV
    FusedArgs fused;             // COEF_FUSED
    void *snap;                  // DUAL: second destination (the next snapshot's payload)
};

// ---------------------------------------------------------------- streaming buffer access
// Every workgroup covers one span (BLOCK lanes x 16 B) of each operand through its own
// buffer descriptor: 32-bit lane offsets whatever the buffer size (7B bf16 = 14 GB), and the
// hardware range check drops the lanes past the end (loads return 0, stores are discarded),
// so no lane branches.  Cache policy, chosen by measurement (tools/lerp_tune.hip,
// profiles/r01b_lerp_tune_*): loads `nt` (each byte is read once per round) and stores `sc1`;
// against plain loads/stores 11.2M fp32 went from 25.4 to 21.6 us cold and from 18.0 to
// 16.4 us Infinity-Cache warm, 100M fp32 from 198 to 189 us.
constexpr int kSpan = kBlock * 16;
// The averaging and publish kernels run one-wave (64-lane) workgroups: inside the gossip
// round (tools/block_sweep.sh, profiles/r01e_block_sweep_*.log) 64 beat 128/256/512 lanes
// cold at 11.2M fp32 (21.7 vs 22.5 us) and at 100M (179-183 vs 182-194 us), and the round
// with a 64-lane publish was the fastest or within noise of it at both sizes.
constexpr int kStreamBlock = 64;
constexpr int kAuxStream = 2;    // nt
constexpr int kAuxStore = 16;    // sc1

template <int SPAN = kSpan>
__device__ __forceinline__ __amdgpu_buffer_rsrc_t span_rsrc(const void *base, int64_t off, int64_t total)
{
    const int64_t rem = total - off;
    const int num = rem <= 0 ? 0 : (rem < SPAN ? (int)rem : SPAN);
    return __builtin_amdgcn_make_buffer_rsrc((void *)((const char *)base + off), 0, num, 0x00020000);
}

template <class V, int AUX = kAuxStream>
__device__ __forceinline__ V span_load(__amdgpu_buffer_rsrc_t r, int lane_off)
{
    return __builtin_bit_cast(V, __builtin_amdgcn_raw_buffer_load_b128(r, lane_off, 0, AUX));
}

template <class V, int AUX = kAuxStore>
__device__ __forceinline__ void span_store(__amdgpu_buffer_rsrc_t r, int lane_off, V v)
{
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, lane_off, 0, AUX);
}

// Cache policies of the averaging kernel (a bit set; the product uses 8, see lerp_policy()):
// the peer snapshot is always read `nt`; the parameters are read `nt` or, with bit 1, with the
// default policy; the result is stored `sc1`, with bit 2 `sc0 sc1`, with bit 4 `nt sc1`.
template <int POLICY> struct LerpPolicy {
    static constexpr int param_load = (POLICY & 1) ? 0 : kAuxStream;
    static constexpr int base_store = kAuxStore | ((POLICY & 2) ? 1 : 0) | ((POLICY & 4) ? kAuxStream : 0);
    // bit 16: only the next snapshot is stored `nt` (a co-resident peer reads it two averages
    // later; this learner's parameters, re-read by its next average one average later, keep
    // the Infinity Cache); bit 32: only the next snapshot is stored `sc0 sc1` (system scope:
    // written through the XCD L2, so the launch's end-of-kernel L2 write-back finds it clean)
    static constexpr int snap_store = base_store | ((POLICY & 16) ? kAuxStream : 0) | ((POLICY & 32) ? 1 : 0);
    // bit 8: the parameters are stored `nt`, leaving the Infinity Cache to the snapshot a peer
    // reads next (the product policy)
    static constexpr int store = base_store | ((POLICY & 8) ? kAuxStream : 0);
};

// Where the peer's bytes are.  ContigSrc: one buffer (a staging buffer, or a peer's slot
// read in place).  StripeSrc: the relay's stripes, stripe s at src[s] (k_lerp_relay).
struct ContigSrc {
    const char *p;
    // byte offset of workgroup b's span: spans in order
    template <int SPAN>
    __device__ __forceinline__ int64_t span_of(uint32_t b) const { return (int64_t)b * SPAN; }
    // base such that base + byte_offset addresses the span starting at span_off
    __device__ __forceinline__ const char *span_base(int64_t) const { return p; }
    __device__ __forceinline__ const char *at(int64_t byte) const { return p + byte; }
};

struct StripeSrc {
    const char *src[kMaxRelayRanks];
    int64_t stripe;    // a multiple of every span (4 KiB multiple): no span straddles stripes
    int32_t parts;     // stripes (ranks)
    // Consecutive workgroups take consecutive stripes (b % parts), so the workgroups in flight
    // at any moment read from every stripe holder -- every xGMI link -- at once, not one
    // stripe (one link) after another.
    template <int SPAN>
    __device__ __forceinline__ int64_t span_of(uint32_t b) const
    {
        return (int64_t)(b % (uint32_t)parts) * stripe + (int64_t)(b / (uint32_t)parts) * SPAN;
    }
    __device__ __forceinline__ const char *span_base(int64_t span_off) const
    {
        const int64_t s = span_off / stripe;
        return src[s] - s * stripe;
    }
    __device__ __forceinline__ const char *at(int64_t byte) const
    {
        const int64_t s = byte / stripe;
        return src[s] + (byte - s * stripe);
    }
};

// One 16-byte item per lane; items beyond n/PER (the ragged tail) go to block 0.
// DUAL also stores the result into args.snap (write-through snapshot: the next publish of
// these parameters then needs no copy).  OOP (with DUAL): the result is stored into args.snap
// ONLY -- the resident form, whose parameters live in the learner's own snapshot slots and move
// from the published slot to the next one at every average (2 reads + 1 write per element, the
// averaging's own bytes; learner.cpp "resident").  BLOCK lanes per workgroup (kStreamBlock).
template <class Ops, int MODE, bool DUAL, int BLOCK, int POLICY, class Src, bool OOP = false>
__device__ __forceinline__ void lerp_span(uint32_t blk, typename Ops::V *__restrict__ param, const Src &src,
                                          int64_t n, const LerpArgs &args)
{
    using V = typename Ops::V;
    constexpr int SPAN = BLOCK * 16;
    const int64_t nv = n / Ops::PER;
    const int64_t span_off = src.template span_of<SPAN>(blk);
    const int lane_off = threadIdx.x * 16;
    const __amdgpu_buffer_rsrc_t rq = span_rsrc<SPAN>(src.span_base(span_off), span_off, nv * 16);
    const __amdgpu_buffer_rsrc_t rp = span_rsrc<SPAN>(param, span_off, nv * 16);
    // issue this lane's loads before anything else
    const V q = span_load<V>(rq, lane_off);
    const V p = span_load<V, LerpPolicy<POLICY>::param_load>(rp, lane_off);
    float a, b;
    if (MODE == COEF_HOST) {
        a = args.a;
        b = args.b;
    } else if (MODE == COEF_DEV) {
        if (args.coef->status != DPWA_STATUS_OK) return;
        a = args.coef->a;
        b = args.coef->b;
    } else {
        bool ok;
        if (BLOCK == 64 && !DPWA_FACTOR_LDS) {
            // one-wave workgroup: every lane evaluates the (uniform) fp64 factor while the loads
            // are in flight and keeps it in registers -- no LDS hand-off, no barrier
            const FusedArgs &fa = args.fused;
            const double loss = read_loss(fa.loss_d, fa.loss_f32, fa.loss_h);
            const dpwa_coef c = factor_math(fa.cfg, *fa.clock_in, fa.hdr->clock, fa.hdr->loss, loss);
            if (blk == 0 && threadIdx.x == 0) factor_commit(fa, c);
            a = c.a;
            b = c.b;
            ok = c.status == DPWA_STATUS_OK;
        } else {
            __shared__ float s_a, s_b;
            __shared__ int s_ok;
            if (threadIdx.x < 64) {  // wave 0: fp64 factor while the loads are in flight
                const FusedArgs &fa = args.fused;
                const double loss = read_loss(fa.loss_d, fa.loss_f32, fa.loss_h);
                const dpwa_coef c = factor_math(fa.cfg, *fa.clock_in, fa.hdr->clock, fa.hdr->loss, loss);
                if (threadIdx.x == 0) {
                    s_a = c.a;
                    s_b = c.b;
                    s_ok = c.status == DPWA_STATUS_OK;
                    if (blk == 0) factor_commit(fa, c);
                }
            }
            __syncthreads();
            a = s_a;
            b = s_b;
            ok = s_ok != 0;
        }
        if (!ok) {            // no-op round; a write-through snapshot still gets the parameters
            if (DUAL)
                span_store<V, LerpPolicy<POLICY>::snap_store>(span_rsrc<SPAN>(args.snap, span_off, nv * 16), lane_off, p);
            if (DUAL && blk == 0 && threadIdx.x < n - nv * Ops::PER) {
                const int64_t j = nv * Ops::PER + threadIdx.x;
                reinterpret_cast<typename Ops::S *>(args.snap)[j] = reinterpret_cast<typename Ops::S *>(param)[j];
            }
            return;
        }
    }
    {
        const V r = Ops::lerp(a, b, q, p);
        if (!OOP) span_store<V, LerpPolicy<POLICY>::store>(rp, lane_off, r);
        if (DUAL) span_store<V, LerpPolicy<POLICY>::snap_store>(span_rsrc<SPAN>(args.snap, span_off, nv * 16), lane_off, r);
    }
    if (blk == 0 && threadIdx.x < n - nv * Ops::PER) {
        using S = typename Ops::S;
        S *ps = reinterpret_cast<S *>(param);
        const int64_t j = nv * Ops::PER + threadIdx.x;
        const S r = Ops::lerp_s(a, b, *reinterpret_cast<const S *>(src.at(j * (int64_t)sizeof(S))), ps[j]);
        if (!OOP) ps[j] = r;
        if (DUAL) reinterpret_cast<S *>(args.snap)[j] = r;
    }
}

template <class Ops, int MODE, bool DUAL, int BLOCK = kBlock, int POLICY = 0, bool OOP = false>
__global__ __launch_bounds__(BLOCK) void k_lerp(typename Ops::V *__restrict__ param,
                                                const typename Ops::V *__restrict__ peer, int64_t n, LerpArgs args)
{
    lerp_span<Ops, MODE, DUAL, BLOCK, POLICY, ContigSrc, OOP>(blockIdx.x, param, ContigSrc{(const char *)peer}, n,
                                                              args);
}

// The relay's fused second phase: the fused average reads the peer's snapshot stripe by stripe
// where the relay left it (stripe s in rank s's relay buffer, the peer's own stripe in its slot,
// ours in local HBM) instead of gathering it into staging first.
template <class Ops, bool DUAL, int POLICY = 0, bool OOP = false>
__global__ __launch_bounds__(kStreamBlock) void k_lerp_relay(typename Ops::V *__restrict__ param, int64_t n,
                                                             LerpArgs args, StripeSrc src)
{
    lerp_span<Ops, COEF_FUSED, DUAL, kStreamBlock, POLICY, StripeSrc, OOP>(blockIdx.x, param, src, n, args);
}

// Several independent fused averages in ONE dispatch (co-resident learners of one round:
// LocalGroup).  Entry i owns the workgroups [begin[i], begin[i+1]); each workgroup runs the
// single-average span code for its entry, so the per-learner semantics (factor, clock commit by
// the entry's first workgroup, ragged tail) are those of k_lerp.  One launch instead of one per
// learner removes a ramp, a drain and a kernel boundary per extra learner.
template <class Ops, bool DUAL, int POLICY = 0, bool OOP = false>
__global__ __launch_bounds__(kStreamBlock) void k_lerp_batch(AvgBatch batch)
{
    int i = 0;
    uint32_t blk;
    if (batch.interleave == 2) {
        // XCD-grouped: workgroup b = (s / 8) * 8E + e * 8 + s % 8 takes span s of entry e, so every
        // entry's span s runs on XCD s % 8 (round-robin dispatch) within a few dispatch slots of the
        // others': entries that read the same buffer -- two resident learners that average with each
        // other both read both published slots -- fetch each span from HBM once, the later reads hit
        // that XCD's L2
        const uint32_t w = 8u * (uint32_t)batch.count;
        const uint32_t r = blockIdx.x % w;
        i = (int)(r >> 3);
        blk = (blockIdx.x / w) * 8u + (r & 7u);
        if (blk >= batch.spans) return;
    } else if (batch.interleave == 1) {
        // entries of equal size, their spans dealt round-robin: a span is read one round after
        // the span at the same position was written by the previous round's dispatch, whichever
        // entry wrote it, so every re-read is equally recent (Infinity Cache residency)
        i = (int)(blockIdx.x % (uint32_t)batch.count);
        blk = blockIdx.x / (uint32_t)batch.count;
    } else {
        // the entry of this workgroup: a short scalar scan over the uniform begin[] table
#pragma unroll
        for (int k = 1; k < kMaxAvgBatch; ++k)
            if (k < batch.count && blockIdx.x >= batch.begin[k]) i = k;
        blk = blockIdx.x - batch.begin[i];
    }
    const AvgEntry &e = batch.e[i];
    LerpArgs args{};
    args.fused = e.fa;
    args.snap = e.snap;
    lerp_span<Ops, COEF_FUSED, DUAL, kStreamBlock, POLICY, ContigSrc, OOP>(blk, (typename Ops::V *)e.param,
                                                                           ContigSrc{(const char *)e.peer}, e.n, args);
}

// A group of resident averages in one pass: co-resident learners whose reads overlap (a slot is
// one learner's parameters and another's peer snapshot, or two learners picked the same peer;
// the N=1 loop's two learners, each the other's only peer, are the mutual pair).  The dispatch's
// U distinct source buffers -- the entries' parameters, then peer snapshots that are no entry's
// parameters -- are loaded once per span by one workgroup, which stores every entry's average
// into its next slot: U loads and `count` stores per lane where the batched span code spends
// 2*count loads (the repeated ones served by L2 at best) over `count` workgroups, and one fp64
// factor evaluation per entry per workgroup as there.  Per entry exactly k_lerp_batch's span
// code: the factor and its commit by workgroup 0, the ZeroDivision no-op (the parameters stored
// unchanged), the ragged tail in workgroup 0.  Entries i < batch.count are src[i]'s averages.
template <class Ops, int POLICY, int U>
__device__ __forceinline__ void group_span(const AvgBatch &batch)
{
    using V = typename Ops::V;
    using S = typename Ops::S;
    using P = LerpPolicy<POLICY>;
    constexpr int SPAN = kStreamBlock * 16;
    const int G = batch.count;       // outputs (<= U), uniform
    const int64_t n = batch.e[0].n;
    const int64_t nv = n / Ops::PER;
    const uint32_t blk = blockIdx.x;
    const int64_t off = (int64_t)blk * SPAN;
    const int lane_off = threadIdx.x * 16;
    V v[U];
#pragma unroll
    for (int j = 0; j < U; ++j)   // all loads first
        v[j] = span_load<V, P::param_load>(span_rsrc<SPAN>(batch.src[j], off, nv * 16), lane_off);
    // per entry: its factor (and workgroup 0's commit), then its average -- one entry's factor
    // live at a time
    float fa_[U], fb_[U];
    bool ok_[U];
    if (DPWA_GROUP_FACTORS_FIRST) {
#pragma unroll
        for (int i = 0; i < U; ++i) {
            if (i >= G) break;
            const FusedArgs &fa = batch.e[i].fa;
            const dpwa_coef c = factor_math(fa.cfg, *fa.clock_in, fa.hdr->clock, fa.hdr->loss,
                                            read_loss(fa.loss_d, fa.loss_f32, fa.loss_h));
            if (blk == 0 && threadIdx.x == 0) factor_commit(fa, c);
            fa_[i] = c.a;
            fb_[i] = c.b;
            ok_[i] = c.status == DPWA_STATUS_OK;
        }
    }
#pragma unroll
    for (int i = 0; i < U; ++i) {
        if (i >= G) break;
        dpwa_coef c;
        if (DPWA_GROUP_FACTORS_FIRST) {
            c.a = fa_[i];
            c.b = fb_[i];
        } else {
            const FusedArgs &fa = batch.e[i].fa;
            c = factor_math(fa.cfg, *fa.clock_in, fa.hdr->clock, fa.hdr->loss, read_loss(fa.loss_d, fa.loss_f32, fa.loss_h));
            if (blk == 0 && threadIdx.x == 0) factor_commit(fa, c);
            fa_[i] = c.a;
            fb_[i] = c.b;
            ok_[i] = c.status == DPWA_STATUS_OK;
        }
        const int k = batch.peer_of[i];   // uniform: a select over registers, no indexed access
        V q = v[0];
#pragma unroll
        for (int j = 1; j < U; ++j)
            if (k == j) q = v[j];
        span_store<V, P::snap_store>(span_rsrc<SPAN>(batch.e[i].snap, off, nv * 16), lane_off,
                                     ok_[i] ? Ops::lerp(c.a, c.b, q, v[i]) : v[i]);
    }
    if (blk == 0 && threadIdx.x < n - nv * Ops::PER) {
        const int64_t j = nv * Ops::PER + threadIdx.x;
        S t[U];
#pragma unroll
        for (int m = 0; m < U; ++m) t[m] = reinterpret_cast<const S *>(batch.src[m])[j];
#pragma unroll
        for (int i = 0; i < U; ++i) {
            if (i >= G) break;
            const int k = batch.peer_of[i];
            S q = t[0];
#pragma unroll
            for (int m = 1; m < U; ++m)
                if (k == m) q = t[m];
            reinterpret_cast<S *>(batch.e[i].snap)[j] = ok_[i] ? Ops::lerp_s(fa_[i], fb_[i], q, t[i]) : t[i];
        }
    }
}

// The mutual pair (two entries, two sources), the N=1 bench's kernel.
template <class Ops, int POLICY>
__global__ __launch_bounds__(kStreamBlock) void k_lerp_pair(AvgBatch batch)
{
    group_span<Ops, POLICY, 2>(batch);
}

// Groups of 3..8 source buffers.
template <class Ops, int POLICY, int U>
__global__ __launch_bounds__(kStreamBlock) void k_lerp_group(AvgBatch batch)
{
    group_span<Ops, POLICY, U>(batch);
}

// Element-wise path for pointers that are not 16-byte aligned (arbitrary views).
template <class Ops, int MODE, bool DUAL>
__global__ __launch_bounds__(kBlock) void k_lerp_unaligned(typename Ops::S *__restrict__ param,
                                                           const typename Ops::S *__restrict__ peer, int64_t n,
                                                           LerpArgs args)
{
    float a, b;
    if (MODE == COEF_HOST) {
        a = args.a;
        b = args.b;
    } else if (MODE == COEF_DEV) {
        if (args.coef->status != DPWA_STATUS_OK) return;
        a = args.coef->a;
        b = args.coef->b;
    } else {
        const FusedArgs &fa = args.fused;
        const double loss = read_loss(fa.loss_d, fa.loss_f32, fa.loss_h);
        const dpwa_coef c = factor_math(fa.cfg, *fa.clock_in, fa.hdr->clock, fa.hdr->loss, loss);
        if (blockIdx.x == 0 && threadIdx.x == 0) factor_commit(fa, c);
        if (c.status != DPWA_STATUS_OK) {
            if (DUAL) {
                const int64_t stride = (int64_t)gridDim.x * kBlock;
                for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride)
                    reinterpret_cast<typename Ops::S *>(args.snap)[i] = param[i];
            }
            return;
        }
        a = c.a;
        b = c.b;
    }
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
        const typename Ops::S r = Ops::lerp_s(a, b, peer[i], param[i]);
        param[i] = r;
        if (DUAL) reinterpret_cast<typename Ops::S *>(args.snap)[i] = r;
    }
}

static inline bool aligned16(const void *p) { return ((uintptr_t)p & 15u) == 0; }

// Workgroup size of the averaging kernel; DPWA_LERP_BLOCK (64/128/256/512) forces another
// (tuning).
static int lerp_block()
{
    static const int forced = [] {
        const char *e = getenv("DPWA_LERP_BLOCK");
        const int b = e ? atoi(e) : 0;
        return (b == 64 || b == 128 || b == 256 || b == 512) ? b : 0;
    }();
    return forced ? forced : kStreamBlock;
}

template <class Ops, int MODE, bool DUAL, int BLOCK, int POLICY = 0>
static hipError_t launch_blocks(void *param, const void *peer, int64_t n, const LerpArgs &args, hipStream_t s,
                                const LaunchTiming *timing)
{
    const int64_t g = (n / Ops::PER) / BLOCK + 1;   // the last span may be empty (range-checked)
    if (timing)   // the dispatch itself is timed (the kernel's begin/end, as a profiler sees it)
        hipExtLaunchKernelGGL((k_lerp<Ops, MODE, DUAL, BLOCK, POLICY>), dim3((uint32_t)g), dim3(BLOCK), 0, s,
                              timing->start, timing->stop, 0, (typename Ops::V *)param,
                              (const typename Ops::V *)peer, n, args);
    else
        hipLaunchKernelGGL((k_lerp<Ops, MODE, DUAL, BLOCK, POLICY>), dim3((uint32_t)g), dim3(BLOCK), 0, s,
                           (typename Ops::V *)param, (const typename Ops::V *)peer, n, args);
    return hipGetLastError();
}

// The product policy is 8 (parameters stored `nt`, the snapshot `sc1`): with the batched
// dispatch it lifts every cold averaging kernel by 1-3 % of peak (11.17M batched 0.78 -> 0.80-0.81,
// 7B bf16 full 0.81 -> 0.82) and leaves the N=1 loop within noise (-0.4 %, two interleaved passes
// with sweeps, profiles/r03_policy_ab.log).  Round 2's one-launch-per-learner loop lost 2-5 % with it
// (profiles/r02_policy_ab2.json).  DPWA_LERP_POLICY overrides (tuning).
constexpr int kProductPolicy = 8;

static int lerp_policy()
{
    static const int forced = [] {
        const char *e = getenv("DPWA_LERP_POLICY");
        const int p = e ? atoi(e) : kProductPolicy;
        return (p >= 0 && p <= 31) ? p : kProductPolicy;
    }();
    return forced;
}

template <class Ops, int MODE, bool DUAL>
static hipError_t launch_mode(void *param, const void *peer, int64_t n, const LerpArgs &args, hipStream_t s,
                              const LaunchTiming *timing)
{
    if (aligned16(param) && aligned16(peer) && aligned16(args.snap)) {
        switch (lerp_block()) {
        case 64:
            switch (lerp_policy()) {
            case 1: return launch_blocks<Ops, MODE, DUAL, 64, 1>(param, peer, n, args, s, timing);
            case 2: return launch_blocks<Ops, MODE, DUAL, 64, 2>(param, peer, n, args, s, timing);
            case 3: return launch_blocks<Ops, MODE, DUAL, 64, 3>(param, peer, n, args, s, timing);
            case 4: return launch_blocks<Ops, MODE, DUAL, 64, 4>(param, peer, n, args, s, timing);
            case 5: return launch_blocks<Ops, MODE, DUAL, 64, 5>(param, peer, n, args, s, timing);
            case 8: return launch_blocks<Ops, MODE, DUAL, 64, 8>(param, peer, n, args, s, timing);
            case 9: return launch_blocks<Ops, MODE, DUAL, 64, 9>(param, peer, n, args, s, timing);
            case 16: return launch_blocks<Ops, MODE, DUAL, 64, 16>(param, peer, n, args, s, timing);
            case 10: return launch_blocks<Ops, MODE, DUAL, 64, 10>(param, peer, n, args, s, timing);
            case 40: return launch_blocks<Ops, MODE, DUAL, 64, 40>(param, peer, n, args, s, timing);
            default: return launch_blocks<Ops, MODE, DUAL, 64>(param, peer, n, args, s, timing);
            }
        // (tuning sizes: the product policy, or policy 0 when DPWA_LERP_POLICY says so)
        case 128:
            return lerp_policy() == kProductPolicy
                       ? launch_blocks<Ops, MODE, DUAL, 128, kProductPolicy>(param, peer, n, args, s, timing)
                       : launch_blocks<Ops, MODE, DUAL, 128>(param, peer, n, args, s, timing);
        case 512:
            return lerp_policy() == kProductPolicy
                       ? launch_blocks<Ops, MODE, DUAL, 512, kProductPolicy>(param, peer, n, args, s, timing)
                       : launch_blocks<Ops, MODE, DUAL, 512>(param, peer, n, args, s, timing);
        default:
            return lerp_policy() == kProductPolicy
                       ? launch_blocks<Ops, MODE, DUAL, 256, kProductPolicy>(param, peer, n, args, s, timing)
                       : launch_blocks<Ops, MODE, DUAL, 256>(param, peer, n, args, s, timing);
        }
    } else {
        // (callers time only the aligned product kernel; an unaligned launch is not timed)
        int64_t g = blocks_for(n);
        if (g > 8192) g = 8192;
        hipLaunchKernelGGL((k_lerp_unaligned<Ops, MODE, DUAL>), dim3((uint32_t)g), dim3(kBlock), 0, s,
                           (typename Ops::S *)param, (const typename Ops::S *)peer, n, args);
    }
    return hipGetLastError();
}

template <class Ops>
static hipError_t launch_ops(int mode, void *param, const void *peer, int64_t n, const LerpArgs &args, hipStream_t s,
                             const LaunchTiming *t)
{
    if (mode == COEF_HOST) return launch_mode<Ops, COEF_HOST, false>(param, peer, n, args, s, t);
    if (mode == COEF_DEV) return launch_mode<Ops, COEF_DEV, false>(param, peer, n, args, s, t);
    if (args.snap) return launch_mode<Ops, COEF_FUSED, true>(param, peer, n, args, s, t);
    return launch_mode<Ops, COEF_FUSED, false>(param, peer, n, args, s, t);
}

static hipError_t launch_any(int32_t dtype, int mode, void *param, const void *peer, int64_t n, const LerpArgs &args,
                             hipStream_t s, const LaunchTiming *t = nullptr)
{
    if (n < 0) return hipErrorInvalidValue;
    if (n == 0 && mode != COEF_FUSED) return hipSuccess;
    if (dtype == DPWA_F32) return launch_ops<OpsF32>(mode, param, peer, n, args, s, t);
    if (dtype == DPWA_BF16) return launch_ops<OpsBF16>(mode, param, peer, n, args, s, t);
    return hipErrorInvalidValue;
}

hipError_t launch_lerp(int32_t dtype, void *param, const void *peer, int64_t n, const dpwa_coef *coef, float a,
                       float b, hipStream_t s)
{
    LerpArgs args{};
    args.a = a;
    args.b = b;
    args.coef = coef;
    return launch_any(dtype, coef ? COEF_DEV : COEF_HOST, param, peer, n, args, s);
}

// The resident form (OOP): one-wave workgroups, the product cache policy unless 0 is forced.
template <class Ops, int POLICY>
static hipError_t launch_oop_policy(void *param, const void *peer, int64_t n, const LerpArgs &args, hipStream_t s,
                                    const LaunchTiming *timing)
{
    const int64_t g = (n / Ops::PER) / kStreamBlock + 1;
    if (timing)
        hipExtLaunchKernelGGL((k_lerp<Ops, COEF_FUSED, true, kStreamBlock, POLICY, true>), dim3((uint32_t)g),
                              dim3(kStreamBlock), 0, s, timing->start, timing->stop, 0, (typename Ops::V *)param,
                              (const typename Ops::V *)peer, n, args);
    else
        hipLaunchKernelGGL((k_lerp<Ops, COEF_FUSED, true, kStreamBlock, POLICY, true>), dim3((uint32_t)g),
                           dim3(kStreamBlock), 0, s, (typename Ops::V *)param, (const typename Ops::V *)peer, n, args);
    return hipGetLastError();
}

// (the resident kernel stores only the next slot, so its store policy is the snapshot one: bit 16
// makes it `nt`, bit 1 loads the parameters with the default policy; tuning variants)
template <class Ops>
static hipError_t launch_oop(void *param, const void *peer, int64_t n, const LerpArgs &args, hipStream_t s,
                             const LaunchTiming *timing)
{
    switch (lerp_policy()) {
    case 0: return launch_oop_policy<Ops, 0>(param, peer, n, args, s, timing);
    case 1: return launch_oop_policy<Ops, 1>(param, peer, n, args, s, timing);
    case 2: return launch_oop_policy<Ops, 2>(param, peer, n, args, s, timing);
    case 16: return launch_oop_policy<Ops, 16>(param, peer, n, args, s, timing);
    case 17: return launch_oop_policy<Ops, 17>(param, peer, n, args, s, timing);
    default: return launch_oop_policy<Ops, kProductPolicy>(param, peer, n, args, s, timing);
    }
}

hipError_t launch_average(int32_t dtype, void *param, const void *peer, int64_t n, const FusedArgs &fa, void *snap,
                          hipStream_t s, const LaunchTiming *timing, bool oop)
{
    LerpArgs args{};
    args.fused = fa;
    args.snap = snap;
    if (oop) {   // resident: 16-B aligned slot payloads only
        if (n < 0 || (!snap && n > 0) || !aligned16(param) || !aligned16(peer) || !aligned16(snap)) return hipErrorInvalidValue;
        if (dtype == DPWA_F32) return launch_oop<OpsF32>(param, peer, n, args, s, timing);
        if (dtype == DPWA_BF16) return launch_oop<OpsBF16>(param, peer, n, args, s, timing);
        return hipErrorInvalidValue;
    }
    return launch_any(dtype, COEF_FUSED, param, peer, n, args, s, timing);
}

// Span order of a batched dispatch of equal-size entries.  Dealt round-robin, every span is
// re-read by the next round's dispatch one round after it was written, which keeps the re-reads
// in the 256 MiB Infinity Cache while a round writes less than that; one entry after the other,
// half the re-reads come 1.5 rounds after their write.  Measured (profiles/r03_batch_order_ab.log,
// three interleaved pairs): round-robin +2.8 % at 11.17M fp32 (179 MB written per round), -4 %
// at 100M fp32 (1.6 GB: twice the concurrent streams, no cache to win).  DPWA_BATCH_ORDER=
// interleaved / contiguous forces one.
constexpr size_t kInfinityCacheBytes = (size_t)256 << 20;

static int batch_order()
{
    static const int forced = [] {
        const char *e = getenv("DPWA_BATCH_ORDER");
        if (e && strcmp(e, "contiguous") == 0) return 0;
        if (e && strcmp(e, "interleaved") == 0) return 1;
        return -1;
    }();
    return forced;
}

// XCD-grouped span order for resident batches whose entries share a read (k_lerp_batch);
// DPWA_BATCH_SHARE=0 turns it off (A/B runs).  tools/pair_tune.hip: two 11.17M fp32 resident
// learners averaging with each other, 36.8 -> 25-27 us per dispatch in the gossip loop, 41.3 ->
// 28.5 us cold (a fused one-workgroup form of both averages: 25.6 / 28.5).
static bool batch_share()
{
    static const bool on = [] {
        const char *e = getenv("DPWA_BATCH_SHARE");
        return !(e && strcmp(e, "0") == 0);
    }();
    return on;
}

// A closed resident group runs as k_lerp_pair / k_lerp_group (one workgroup per span for all its
// averages); DPWA_PAIR_FUSED=0 keeps it on the XCD-grouped batch (A/B runs).
static bool pair_fused()
{
    static const bool on = [] {
        const char *e = getenv("DPWA_PAIR_FUSED");
        return !(e && strcmp(e, "0") == 0);
    }();
    return on;
}

// Some buffer is read by two entries (as parameters or as the peer snapshot).
static bool shares_a_read(const AvgBatch &x)
{
    for (int i = 0; i < x.count; ++i)
        for (int j = 0; j < x.count; ++j)
            if (i != j && (x.e[i].peer == x.e[j].param || (j > i && x.e[i].peer == x.e[j].peer)))
                return true;
    return false;
}

hipError_t launch_average_batch(int32_t dtype, bool dual, const AvgBatch &b, hipStream_t s,
                                 const LaunchTiming *timing, bool oop)
{
    if (b.count < 1 || b.count > kMaxAvgBatch || (oop && !dual)) return hipErrorInvalidValue;
    AvgBatch x = b;
    uint32_t g = 0;
    const int per = dtype == DPWA_F32 ? OpsF32::PER : dtype == DPWA_BF16 ? OpsBF16::PER : 0;
    if (!per) return hipErrorInvalidValue;
    for (int i = 0; i < x.count; ++i) {
        const AvgEntry &e = x.e[i];
        if (e.n < 0 || !aligned16(e.param) || !aligned16(e.peer) || (!dual && e.snap) || (dual && !e.snap && e.n > 0) ||
            !aligned16(e.snap))
            return hipErrorInvalidValue;
        const int64_t gi = (e.n / per) / kStreamBlock + 1;   // as launch_blocks: last span may be empty
        if (gi > 0x7fffffffLL) return hipErrorInvalidValue;
    }
    int64_t total = 0;   // in 64 bits: up to 8 entries of up to 2^31 - 1 workgroups each
    for (int i = 0; i < x.count; ++i) {
        x.begin[i] = (uint32_t)total;
        total += (x.e[i].n / per) / kStreamBlock + 1;
        if (total > 0x7fffffffLL) return hipErrorInvalidValue;
    }
    g = (uint32_t)total;
    for (int i = x.count; i < kMaxAvgBatch; ++i) x.begin[i] = 0xffffffffu;
    // span order: see batch_order()
    bool same = true;
    size_t written = 0;
    for (int i = 0; i < x.count; ++i) {
        same = same && x.e[i].n == x.e[0].n;
        written += (size_t)x.e[i].n * (size_t)(per == OpsF32::PER ? 4 : 2) * (dual && !oop ? 2 : 1);
    }
    const int order = batch_order();
    x.interleave = same && x.count > 1 && (order == 1 || (order < 0 && written <= kInfinityCacheBytes)) ? 1 : 0;
    // resident entries of equal size that read a common buffer (a learner's published slot is its
    // own parameters and another's peer): XCD-grouped, whatever the size (nothing writes what they
    // read, so any order is safe)
    x.spans = (uint32_t)((x.e[0].n / per) / kStreamBlock + 1);
    // a group: entries of equal size, distinct parameters, whose reads overlap; its sources are
    // the parameters, then the peers that are no entry's parameters (at most kMaxAvgBatch)
    bool grouped = oop && same && x.count > 1 && order < 0 && batch_share() && pair_fused();
    int nsrc = x.count;
    for (int i = 0; grouped && i < x.count; ++i) {
        x.src[i] = x.e[i].param;
        for (int j = 0; j < i; ++j)
            if (x.e[j].param == x.e[i].param) grouped = false;
    }
    for (int i = 0; grouped && i < x.count; ++i) {
        int k = -1;
        for (int j = 0; j < nsrc && k < 0; ++j)
            if (x.src[j] == x.e[i].peer) k = j;
        if (k < 0) {
            if (nsrc == kMaxAvgBatch) grouped = false;
            else {
                k = nsrc;
                x.src[nsrc++] = x.e[i].peer;
            }
        }
        x.peer_of[i] = (int8_t)k;
        grouped = grouped && k != i;
    }
    grouped = grouped && nsrc < 2 * x.count;   // some read is shared
    for (int j = nsrc; j < kMaxAvgBatch; ++j) x.src[j] = nullptr;
    const bool closed = grouped && nsrc == 2 && x.count == 2;   // the mutual pair
    if (grouped && !closed) {
#define DPWA_GROUP_LAUNCH(OPS, P, G)                                                                         \
    do {                                                                                                    \
        if (timing)                                                                                         \
            hipExtLaunchKernelGGL((k_lerp_group<OPS, P, G>), dim3(x.spans), dim3(kStreamBlock), 0, s,        \
                                  timing->start, timing->stop, 0, x);                                       \
        else                                                                                                \
            hipLaunchKernelGGL((k_lerp_group<OPS, P, G>), dim3(x.spans), dim3(kStreamBlock), 0, s, x);     \
    } while (0)
#define DPWA_GROUP_G(OPS, P)                                                                                 \
    do {                                                                                                    \
        switch (nsrc) {                                                                                     \
        case 3: DPWA_GROUP_LAUNCH(OPS, P, 3); break;                                                        \
        case 4: DPWA_GROUP_LAUNCH(OPS, P, 4); break;                                                        \
        case 5: DPWA_GROUP_LAUNCH(OPS, P, 5); break;                                                        \
        case 6: DPWA_GROUP_LAUNCH(OPS, P, 6); break;                                                        \
        case 7: DPWA_GROUP_LAUNCH(OPS, P, 7); break;                                                        \
        default: DPWA_GROUP_LAUNCH(OPS, P, 8); break;                                                       \
        }                                                                                                   \
    } while (0)
        const bool p0 = lerp_policy() == 0;
        if (dtype == DPWA_F32) {
            if (p0) DPWA_GROUP_G(OpsF32, 0);
            else DPWA_GROUP_G(OpsF32, kProductPolicy);
        } else {
            if (p0) DPWA_GROUP_G(OpsBF16, 0);
            else DPWA_GROUP_G(OpsBF16, kProductPolicy);
        }
#undef DPWA_GROUP_G
#undef DPWA_GROUP_LAUNCH
        return hipGetLastError();
    }
    if (closed) {
        // a mutual pair: both averages in one workgroup per span
#define DPWA_PAIR_LAUNCH(OPS, P)                                                                             \
    do {                                                                                                    \
        if (timing)                                                                                         \
            hipExtLaunchKernelGGL((k_lerp_pair<OPS, P>), dim3(x.spans), dim3(kStreamBlock), 0, s,            \
                                  timing->start, timing->stop, 0, x);                                       \
        else                                                                                                \
            hipLaunchKernelGGL((k_lerp_pair<OPS, P>), dim3(x.spans), dim3(kStreamBlock), 0, s, x);         \
    } while (0)
        // cache-policy variants for tuning (DPWA_LERP_POLICY); both loads take the parameter load's
        // policy (each slot is one entry's parameters and the other's peer)
        if (dtype == DPWA_F32) {
            switch (lerp_policy()) {
            case 0: DPWA_PAIR_LAUNCH(OpsF32, 0); break;
            case 1: DPWA_PAIR_LAUNCH(OpsF32, 1); break;
            case 2: DPWA_PAIR_LAUNCH(OpsF32, 2); break;
            case 16: DPWA_PAIR_LAUNCH(OpsF32, 16); break;
            case 32: DPWA_PAIR_LAUNCH(OpsF32, 32); break;
            default: DPWA_PAIR_LAUNCH(OpsF32, kProductPolicy); break;
            }
        } else {
            if (lerp_policy() == 0) DPWA_PAIR_LAUNCH(OpsBF16, 0);
            else DPWA_PAIR_LAUNCH(OpsBF16, kProductPolicy);
        }
#undef DPWA_PAIR_LAUNCH
        return hipGetLastError();
    }
    if (oop && same && x.count > 1 && order < 0 && batch_share() && shares_a_read(x)) {
        const uint64_t gg = (uint64_t)(x.spans + 7) / 8 * 8 * (uint64_t)x.count;
        if (gg > 0x7fffffffu) return hipErrorInvalidValue;
        x.interleave = 2;
        g = (uint32_t)gg;
    }
#define DPWA_BATCH_LAUNCH_P(OPS, DL, P, OOP)                                                                \
    do {                                                                                                    \
        if (timing)                                                                                         \
            hipExtLaunchKernelGGL((k_lerp_batch<OPS, DL, P, OOP>), dim3(g), dim3(kStreamBlock), 0, s,        \
                                  timing->start, timing->stop, 0, x);                                       \
        else                                                                                                \
            hipLaunchKernelGGL((k_lerp_batch<OPS, DL, P, OOP>), dim3(g), dim3(kStreamBlock), 0, s, x);     \
    } while (0)
    // cache-policy variants for tuning (DPWA_LERP_POLICY, as the single-learner kernel)
#define DPWA_BATCH_LAUNCH(OPS, DL)                                                                          \
    do {                                                                                                    \
        switch (lerp_policy()) {                                                                            \
        case 1: DPWA_BATCH_LAUNCH_P(OPS, DL, 1, false); break;                                              \
        case 2: DPWA_BATCH_LAUNCH_P(OPS, DL, 2, false); break;                                              \
        case 8: DPWA_BATCH_LAUNCH_P(OPS, DL, 8, false); break;                                              \
        case 9: DPWA_BATCH_LAUNCH_P(OPS, DL, 9, false); break;                                              \
        case 16: DPWA_BATCH_LAUNCH_P(OPS, DL, 16, false); break;                                            \
        case 10: DPWA_BATCH_LAUNCH_P(OPS, DL, 10, false); break;                                            \
        case 40: DPWA_BATCH_LAUNCH_P(OPS, DL, 40, false); break;                                            \
        default: DPWA_BATCH_LAUNCH_P(OPS, DL, 0, false); break;                                             \
        }                                                                                                   \
    } while (0)
    // the resident form: the product policy unless 0 is forced
#define DPWA_BATCH_LAUNCH_OOP(OPS)                                                                          \
    do {                                                                                                    \
        switch (lerp_policy()) {                                                                            \
        case 0: DPWA_BATCH_LAUNCH_P(OPS, true, 0, true); break;                                             \
        case 1: DPWA_BATCH_LAUNCH_P(OPS, true, 1, true); break;                                             \
        case 2: DPWA_BATCH_LAUNCH_P(OPS, true, 2, true); break;                                             \
        case 16: DPWA_BATCH_LAUNCH_P(OPS, true, 16, true); break;                                           \
        case 17: DPWA_BATCH_LAUNCH_P(OPS, true, 17, true); break;                                           \
        default: DPWA_BATCH_LAUNCH_P(OPS, true, kProductPolicy, true); break;                               \
        }                                                                                                   \
    } while (0)
    if (dtype == DPWA_F32) {
        if (oop) DPWA_BATCH_LAUNCH_OOP(OpsF32);
        else if (dual) DPWA_BATCH_LAUNCH(OpsF32, true);
        else DPWA_BATCH_LAUNCH(OpsF32, false);
    } else {
        if (oop) DPWA_BATCH_LAUNCH_OOP(OpsBF16);
        else if (dual) DPWA_BATCH_LAUNCH(OpsBF16, true);
        else DPWA_BATCH_LAUNCH(OpsBF16, false);
    }
#undef DPWA_BATCH_LAUNCH_OOP
#undef DPWA_BATCH_LAUNCH
#undef DPWA_BATCH_LAUNCH_P
    return hipGetLastError();
}

__global__ void k_acquire_system();

template <class Ops, bool DUAL, int POLICY, bool OOP>
static void launch_relay_policy(void *param, int64_t n, const LerpArgs &args, const StripeSrc &src, hipStream_t s,
                                const LaunchTiming *timing)
{
    // every span of every stripe (the spans past the payload are range-checked away)
    const int64_t g = (int64_t)src.parts * (src.stripe / (kStreamBlock * 16));
    if (timing)
        hipExtLaunchKernelGGL((k_lerp_relay<Ops, DUAL, POLICY, OOP>), dim3((uint32_t)g), dim3(kStreamBlock), 0, s,
                              timing->start, timing->stop, 0, (typename Ops::V *)param, n, args, src);
    else
        hipLaunchKernelGGL((k_lerp_relay<Ops, DUAL, POLICY, OOP>), dim3((uint32_t)g), dim3(kStreamBlock), 0, s,
                           (typename Ops::V *)param, n, args, src);
}

// the product cache policy (lerp_policy(): local parameters stored nt) or, forced to 0, the old one
template <class Ops, bool DUAL, bool OOP = false>
static void launch_relay_kernel(void *param, int64_t n, const LerpArgs &args, const StripeSrc &src, hipStream_t s,
                                const LaunchTiming *timing)
{
    if (lerp_policy() == 8) launch_relay_policy<Ops, DUAL, 8, OOP>(param, n, args, src, s, timing);
    else launch_relay_policy<Ops, DUAL, 0, OOP>(param, n, args, src, s, timing);
}

hipError_t launch_average_relay(int32_t dtype, void *param, int64_t n, const FusedArgs &fa, void *snap,
                                const RelayArgs &a, int my_pick, hipStream_t s, const LaunchTiming *timing, bool oop)
{
    if (n < 0 || a.world < 1 || a.world > kMaxRelayRanks || my_pick < 0 || my_pick >= a.world ||
        my_pick == a.rank || a.stripe <= 0 || a.stripe % (kStreamBlock * 16) || !aligned16(param) ||
        (snap && !aligned16(snap)) || (oop && !snap))
        return hipErrorInvalidValue;
    const int j = my_pick;
    StripeSrc src;
    for (int r = 0; r < a.world; ++r)   // where stripe r of j's snapshot is (k_relay_phase2's sources)
        src.src[r] = r == j        ? a.slots[j] + a.slot_off + DPWA_SLOT_PAYLOAD_OFFSET + (int64_t)r * a.stripe
                     : r == a.rank ? a.relay_mine + (int64_t)j * a.stripe
                                   : a.relays[r] + (int64_t)j * a.stripe;
    for (int r = a.world; r < kMaxRelayRanks; ++r) src.src[r] = nullptr;
    src.stripe = a.stripe;
    src.parts = a.world;
    LerpArgs args{};
    args.fused = fa;
    args.snap = snap;
    hipLaunchKernelGGL(k_acquire_system, dim3(256), dim3(64), 0, s);   // remote lines in L2 are stale
    if (dtype == DPWA_F32) {
        if (oop) launch_relay_kernel<OpsF32, true, true>(param, n, args, src, s, timing);
        else if (snap) launch_relay_kernel<OpsF32, true>(param, n, args, src, s, timing);
        else launch_relay_kernel<OpsF32, false>(param, n, args, src, s, timing);
    } else if (dtype == DPWA_BF16) {
        if (oop) launch_relay_kernel<OpsBF16, true, true>(param, n, args, src, s, timing);
        else if (snap) launch_relay_kernel<OpsBF16, true>(param, n, args, src, s, timing);
        else launch_relay_kernel<OpsBF16, false>(param, n, args, src, s, timing);
    } else {
        return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// ---------------------------------------------------------------- publish
template <bool VEC, int BLOCK = kBlock>
__global__ __launch_bounds__(BLOCK) void k_publish(char *__restrict__ slot, const char *__restrict__ flat,
                                                   int64_t nbytes, int64_t n, int32_t dtype,
                                                   double *__restrict__ clock, double loss_h,
                                                   const double *__restrict__ loss_d, int32_t loss_f32,
                                                   uint64_t version)
{
    char *payload = slot + DPWA_SLOT_PAYLOAD_OFFSET;
    if (VEC) {   // one 16-B item per lane, streaming policy of the lerp (nt loads, sc1 stores)
        constexpr int SPAN = BLOCK * 16;
        const int64_t n16 = nbytes >> 4;
        const int64_t span_off = (int64_t)blockIdx.x * SPAN;
        const int lane_off = threadIdx.x * 16;
        span_store(span_rsrc<SPAN>(payload, span_off, n16 * 16), lane_off,
                   span_load<u32x4>(span_rsrc<SPAN>(flat, span_off, n16 * 16), lane_off));
        if (blockIdx.x == 0 && threadIdx.x < (nbytes & 15)) {
            const int64_t j = (n16 << 4) + threadIdx.x;
            payload[j] = flat[j];
        }
    } else {
        const int64_t stride = (int64_t)gridDim.x * kBlock;
        for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < nbytes; i += stride) payload[i] = flat[i];
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        dpwa_header *h = reinterpret_cast<dpwa_header *>(slot);
        const double c = *clock + 1.0;                 // dpwa.py:112  self.clock += 1
        *clock = c;
        h->clock = c;                                  // dpwa.py:115  state = {'clock', 'loss'}
        h->loss = read_loss(loss_d, loss_f32, loss_h);
        h->version = version;
        h->n = n;
        h->dtype = dtype;
    }
}

// Local streaming copy of a payload (a resident learner's relocation: the parameters leave the
// published slot for the next one), the publish's span shape without the header.
template <int BLOCK>
__global__ __launch_bounds__(BLOCK) void k_copy_payload(char *__restrict__ dst, const char *__restrict__ src,
                                                        int64_t nbytes)
{
    constexpr int SPAN = BLOCK * 16;
    const int64_t n16 = nbytes >> 4;
    const int64_t span_off = (int64_t)blockIdx.x * SPAN;
    const int lane_off = threadIdx.x * 16;
    span_store(span_rsrc<SPAN>(dst, span_off, n16 * 16), lane_off,
               span_load<u32x4>(span_rsrc<SPAN>(src, span_off, n16 * 16), lane_off));
    if (blockIdx.x == 0 && threadIdx.x < (nbytes & 15)) {
        const int64_t j = (n16 << 4) + threadIdx.x;
        dst[j] = src[j];
    }
}

hipError_t launch_copy_payload(void *dst, const void *src, int64_t nbytes, hipStream_t s)
{
    if (nbytes <= 0) return hipSuccess;
    if (!aligned16(dst) || !aligned16(src))
        return hipMemcpyAsync(dst, src, (size_t)nbytes, hipMemcpyDeviceToDevice, s);
    const int64_t g = (nbytes >> 4) / kStreamBlock + 1;
    if (g > 0x7fffffffLL) return hipMemcpyAsync(dst, src, (size_t)nbytes, hipMemcpyDeviceToDevice, s);
    hipLaunchKernelGGL(k_copy_payload<kStreamBlock>, dim3((uint32_t)g), dim3(kStreamBlock), 0, s, (char *)dst,
                       (const char *)src, nbytes);
    return hipGetLastError();
}

// Pull: copy a peer's snapshot (header + payload, IPC-mapped in another GPU's HBM) into the
// local staging buffer.  The loads travel over the xGMI link to the owner; each lane keeps
// four 16-byte loads in flight and the grid is capped (grid-stride) so the pull occupies a
// bounded share of the CUs while the training step runs on the compute stream.
__global__ __launch_bounds__(kBlock) void k_pull(u32x4 *__restrict__ dst, const u32x4 *__restrict__ src, int64_t n16)
{
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    for (; i + 3 * stride < n16; i += 4 * stride) {
        u32x4 v0 = src[i], v1 = src[i + stride], v2 = src[i + 2 * stride], v3 = src[i + 3 * stride];
        dst[i] = v0;
        dst[i + stride] = v1;
        dst[i + 2 * stride] = v2;
        dst[i + 3 * stride] = v3;
    }
    for (; i < n16; i += stride) dst[i] = src[i];
}

// Invalidates every XCD's L2 lines of other agents' memory (system-scope acquire from 256
// workgroups, dealt round-robin over the 8 XCDs) ahead of a kernel that reads peer memory.
__global__ __launch_bounds__(64) void k_acquire_system()
{
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
}

hipError_t launch_pull(void *dst, const void *src, int64_t nbytes, int max_blocks, bool remote, hipStream_t s)
{
    if (((uintptr_t)dst | (uintptr_t)src | (uintptr_t)nbytes) & 15) return hipErrorInvalidValue;
    if (remote) hipLaunchKernelGGL(k_acquire_system, dim3(256), dim3(64), 0, s);
    const int64_t n16 = nbytes >> 4;
    int64_t g = (n16 + kBlock * 4 - 1) / (kBlock * 4);
    if (g < 1) g = 1;
    if (g > max_blocks) g = max_blocks;
    hipLaunchKernelGGL(k_pull, dim3((uint32_t)g), dim3(kBlock), 0, s, (u32x4 *)dst, (const u32x4 *)src, n16);
    return hipGetLastError();
}

// ---------------------------------------------------------------- relay (multi-link pull)
// Lock-step round of G ranks where rank i averages with rank picks[i] (-1: none).  Each
// snapshot payload is cut into G stripes.  Phase 1 on rank r pulls stripe r of every
// snapshot some rank needs (its own peer's included) into its relay buffer (R_r[j] = stripe
// r of rank j); after a barrier, phase 2 on rank r gathers stripe s of its peer j's snapshot
// from rank s's relay buffer, from its own relay buffer for s == r (local HBM) and from j
// itself for s == j.  Every pair's xGMI link then carries at most one stripe per phase
// instead of one link carrying the whole snapshot.
// blockIdx.x selects the source (phase 1) or the stripe (phase 2) and blockIdx.y strides it:
// consecutive workgroups (the dispatch order) take different sources, so every link is busy
// from the start even when the grid exceeds what is resident at once.
__global__ void k_release_system();

__device__ __forceinline__ void copy16(u32x4 *__restrict__ dst, const u32x4 *__restrict__ src, int64_t n16)
{
    const int64_t stride = (int64_t)gridDim.y * kBlock;
    int64_t i = (int64_t)blockIdx.y * kBlock + threadIdx.x;
    for (; i + 3 * stride < n16; i += 4 * stride) {
        u32x4 v0 = src[i], v1 = src[i + stride], v2 = src[i + 2 * stride], v3 = src[i + 3 * stride];
        dst[i] = v0;
        dst[i + stride] = v1;
        dst[i + 2 * stride] = v2;
        dst[i + 3 * stride] = v3;
    }
    for (; i < n16; i += stride) dst[i] = src[i];
}

__device__ __forceinline__ int64_t stripe_len(int s, int64_t stripe, int64_t payload)
{
    const int64_t beg = (int64_t)s * stripe;
    if (beg >= payload) return 0;
    return (payload - beg < stripe ? payload - beg : stripe);
}

__global__ __launch_bounds__(kBlock) void k_relay_phase1(RelayArgs a)
{
    const int j = blockIdx.x;
    if (j == a.rank) return;
    bool active = false;                                   // does any rank (me included) need j?
    for (int i = 0; i < a.world; ++i) active |= (a.picks[i] == j);
    if (!active) return;
    const int64_t len = stripe_len(a.rank, a.stripe, a.payload);
    const char *src = a.slots[j] + a.slot_off + DPWA_SLOT_PAYLOAD_OFFSET + (int64_t)a.rank * a.stripe;
    char *dst = a.relay_mine + (int64_t)j * a.stripe;
    copy16((u32x4 *)dst, (const u32x4 *)src, len >> 4);
}

__global__ __launch_bounds__(kBlock) void k_relay_phase2(RelayArgs a)
{
    const int j = a.picks[a.rank];
    if (j < 0) return;
    const int s = blockIdx.x;
    if (s == 0 && blockIdx.y == 0 && threadIdx.x < 16)     // the 256-B header, straight from j
        reinterpret_cast<u32x4 *>(a.staging)[threadIdx.x] =
            reinterpret_cast<const u32x4 *>(a.slots[j] + a.slot_off)[threadIdx.x];
    const int64_t len = stripe_len(s, a.stripe, a.payload);
    const char *src = s == j        ? a.slots[j] + a.slot_off + DPWA_SLOT_PAYLOAD_OFFSET + (int64_t)s * a.stripe
                      : s == a.rank ? a.relay_mine + (int64_t)j * a.stripe
                                    : a.relays[s] + (int64_t)j * a.stripe;
    copy16((u32x4 *)(a.staging + DPWA_SLOT_PAYLOAD_OFFSET + (int64_t)s * a.stripe), (const u32x4 *)src, len >> 4);
}

hipError_t launch_relay(int phase, const RelayArgs &a, int blocks_per_part, hipStream_t s)
{
    if (a.world < 1 || a.world > kMaxRelayRanks || (a.stripe & 15) || (a.payload & 15)) return hipErrorInvalidValue;
    dim3 grid((uint32_t)a.world, (uint32_t)blocks_per_part);
    hipLaunchKernelGGL(k_acquire_system, dim3(256), dim3(64), 0, s);   // both phases read peers
    if (phase == 1) {   // the relay buffer is read by other GPUs: write it back from the L2s
        hipLaunchKernelGGL(k_relay_phase1, grid, dim3(kBlock), 0, s, a);
        hipLaunchKernelGGL(k_release_system, dim3(256), dim3(64), 0, s);
    } else {
        hipLaunchKernelGGL(k_relay_phase2, grid, dim3(kBlock), 0, s, a);
    }
    return hipGetLastError();
}

// Writes back every XCD's L2 (system-scope release from 256 workgroups, which the
// dispatcher deals round-robin over the 8 XCDs) so a snapshot that another GPU will pull
// is in HBM, not only in this GPU's L2s.  Used only once the slots are IPC-exported.
__global__ __launch_bounds__(64) void k_release_system()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
}

hipError_t launch_release_system(hipStream_t s)
{
    hipLaunchKernelGGL(k_release_system, dim3(256), dim3(64), 0, s);
    return hipGetLastError();
}

// Workgroup size of the snapshot copy; DPWA_PUBLISH_BLOCK (64/128/256) forces another.
static int publish_block()
{
    static const int forced = [] {
        const char *e = getenv("DPWA_PUBLISH_BLOCK");
        const int b = e ? atoi(e) : 0;
        return (b == 64 || b == 128 || b == 256) ? b : 0;
    }();
    return forced ? forced : kStreamBlock;
}

hipError_t launch_publish(char *slot, const void *flat, int64_t nbytes, int64_t n, int32_t dtype, double *clock,
                          double loss, const double *loss_dev, bool loss_f32, uint64_t version, bool system_release,
                          hipStream_t s)
{
    const char *src = (const char *)flat;
    if (aligned16(flat)) {
        const int64_t n16 = nbytes >> 4;
        const int b = publish_block();
        const int64_t g = n16 / b + 1;
        if (b == 64)
            hipLaunchKernelGGL((k_publish<true, 64>), dim3((uint32_t)g), dim3(64), 0, s, slot, src, nbytes, n, dtype,
                               clock, loss, loss_dev, (int32_t)loss_f32, version);
        else if (b == 128)
            hipLaunchKernelGGL((k_publish<true, 128>), dim3((uint32_t)g), dim3(128), 0, s, slot, src, nbytes, n,
                               dtype, clock, loss, loss_dev, (int32_t)loss_f32, version);
        else
            hipLaunchKernelGGL((k_publish<true>), dim3((uint32_t)g), dim3(kBlock), 0, s, slot, src, nbytes, n, dtype,
                               clock, loss, loss_dev, (int32_t)loss_f32, version);
    } else {
        int64_t g = blocks_for(nbytes);
        if (g > 8192) g = 8192;
        hipLaunchKernelGGL((k_publish<false>), dim3((uint32_t)g), dim3(kBlock), 0, s, slot, src, nbytes, n, dtype,
                           clock, loss, loss_dev, (int32_t)loss_f32, version);
    }
    if (system_release) hipLaunchKernelGGL(k_release_system, dim3(256), dim3(64), 0, s);
    return hipGetLastError();
}

// Header-only publish: the payload of `slot` was already written by a write-through
// average of exactly these parameters.
__global__ void k_publish_header(char *__restrict__ slot, int64_t n, int32_t dtype, double *__restrict__ clock,
                                 double loss_h, const double *__restrict__ loss_d, int32_t loss_f32, uint64_t version)
{
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    dpwa_header *h = reinterpret_cast<dpwa_header *>(slot);
    const double c = *clock + 1.0;                     // dpwa.py:112
    *clock = c;
    h->clock = c;
    h->loss = read_loss(loss_d, loss_f32, loss_h);
    h->version = version;
    h->n = n;
    h->dtype = dtype;
}

hipError_t launch_publish_header(char *slot, int64_t n, int32_t dtype, double *clock, double loss,
                                 const double *loss_dev, bool loss_f32, uint64_t version, bool system_release,
                                 hipStream_t s)
{
    hipLaunchKernelGGL(k_publish_header, dim3(1), dim3(64), 0, s, slot, n, dtype, clock, loss, loss_dev, (int32_t)loss_f32, version);
    if (system_release) hipLaunchKernelGGL(k_release_system, dim3(256), dim3(64), 0, s);
    return hipGetLastError();
}

// Reuse guard of a header-only publish (the adapter's write-through): writes
// through `param.data` move no version counter, so before a snapshot the last average wrote is
// published as is, the parameters are compared with it at kGuardSamples 16-B words, and what
// differs is copied.  The payload is cut into kGuardSamples chunks, chunk k = words [b(k), b(k+1))
// with b(k) = k (n16-1) / (samples-1) (the last chunk is the last word alone); chunk k is sampled
// at one word, b(k) + gen mod (its length), so the sampled word moves on by one each publish and
// every word of the parameters is compared once in any W = ceil((n16-1)/4095) publishes -- a
// sparse write through `param.data` that one publish's samples miss is published within W
// publishes, at the same per-publish cost.  The first word (and the tail bytes) are compared at
// every publish too.  A chunk whose sample differs is copied from the parameters into the
// payload by the workgroup that sampled it, so one launch does the check and the copy: no
// verdict has to reach other workgroups (round 5 ran a compare and a grid-wide conditional copy
// as two launches).  A workgroup that finds a difference stamps the verdict word with this
// publish's generation `gen` (never cleared; the first stamp of a generation counts a hit).
constexpr int kGuardSamples = 4096;
constexpr int kGuardWave = 64;
constexpr int kGuardChunksPerBlock = 16;     // chunks sampled by one workgroup (lanes 0..15 of wave 0)
constexpr int kGuardBlock = 256;             // 4 waves copy a dirty chunk

// b(k) = k (n16-1) / (samples-1).  samples = min(n16, kGuardSamples): below kGuardSamples words it
// is k itself, otherwise the divisor is the constant kGuardSamples-1, which compiles to a
// multiply-high -- the sampling lanes' addresses wait on this, and a 64-bit division by a
// variable is a long emulated sequence on the VALU.
__device__ __forceinline__ int64_t guard_base(int64_t k, int64_t samples, int64_t n16)
{
    if (samples <= 1) return 0;
    if (samples < kGuardSamples) return k;
    return (int64_t)((uint64_t)k * (uint64_t)(n16 - 1) / (uint64_t)(kGuardSamples - 1));
}

// Byte offset of the word sampled in chunk k (of `samples`) over n16 16-B words at generation `gen`.
__device__ __forceinline__ int64_t guard_offset(int64_t k, int64_t samples, int64_t n16, uint32_t gen)
{
    if (samples <= 1 || k >= samples - 1) return (samples > 1 ? n16 - 1 : 0) << 4;
    const int64_t b = guard_base(k, samples, n16);
    const int64_t len = guard_base(k + 1, samples, n16) - b;        // >= 1
    const int64_t r = len <= (int64_t)UINT32_MAX ? (int64_t)(gen % (uint32_t)len) : (int64_t)(gen % (uint64_t)len);
    return (b + r) << 4;
}

__global__ __launch_bounds__(kGuardBlock) void k_guard_publish(const char *__restrict__ flat,
                                                               char *__restrict__ payload, int64_t nbytes,
                                                               int32_t *__restrict__ dirty,
                                                               uint32_t *__restrict__ hits, int32_t gen)
{
    __shared__ uint32_t s_mask;
    const int64_t n16 = nbytes >> 4;
    const int64_t samples = n16 < kGuardSamples ? n16 : kGuardSamples;
    const int64_t k0 = (int64_t)blockIdx.x * kGuardChunksPerBlock;
    const int t = threadIdx.x;
    if (t < kGuardWave) {
        int diff = 0;
        const int64_t k = k0 + t;
        if (t < kGuardChunksPerBlock && k < samples) {
            const int64_t o = guard_offset(k, samples, n16, (uint32_t)gen);
            const u32x4 a = *reinterpret_cast<const u32x4 *>(flat + o);
            const u32x4 b = *reinterpret_cast<const u32x4 *>(payload + o);
            diff = (a.x != b.x) | (a.y != b.y) | (a.z != b.z) | (a.w != b.w);
        }
        if (blockIdx.x == 0 && t == kGuardChunksPerBlock && n16 > 0) {   // the first word, always: chunk 0
            const u32x4 a = *reinterpret_cast<const u32x4 *>(flat);
            const u32x4 b = *reinterpret_cast<const u32x4 *>(payload);
            if ((a.x != b.x) | (a.y != b.y) | (a.z != b.z) | (a.w != b.w)) diff = 1;
        }
        // bit c: chunk k0 + c differs (the first-word lane reports chunk 0)
        const uint64_t ballot = __ballot(diff);
        uint32_t mask = (uint32_t)(ballot & ((1u << kGuardChunksPerBlock) - 1u));
        if (ballot >> kGuardChunksPerBlock) mask |= 1u;
        if (t == 0) s_mask = mask;
    }
    // the tail bytes (past the last whole word) belong to workgroup 0: compared and copied in place
    int tail_diff = 0;
    if (blockIdx.x == 0 && t >= kGuardWave && t < kGuardWave + (nbytes & 15)) {
        const int64_t j = (n16 << 4) + (t - kGuardWave);
        if (flat[j] != payload[j]) {
            payload[j] = flat[j];
            tail_diff = 1;
        }
    }
    tail_diff = __syncthreads_or(tail_diff);
    const uint32_t mask = s_mask;
    if ((mask || tail_diff) && t == 0) {
        const int32_t old = atomicExch(dirty, gen);
        if (old != gen) atomicAdd(hits, 1u);
    }
    for (uint32_t m = mask; m; m &= m - 1) {
        const int64_t k = k0 + __builtin_ctz(m);
        const int64_t lo = k >= samples - 1 ? (samples > 1 ? n16 - 1 : 0) : guard_base(k, samples, n16);
        const int64_t hi = k >= samples - 1 ? n16 : guard_base(k + 1, samples, n16);
        u32x4 *d = reinterpret_cast<u32x4 *>(payload);
        const u32x4 *src = reinterpret_cast<const u32x4 *>(flat);
        int64_t i = lo + t;
        for (; i + 3 * kGuardBlock < hi; i += 4 * kGuardBlock) {   // four loads in flight per lane
            const u32x4 v0 = src[i], v1 = src[i + kGuardBlock], v2 = src[i + 2 * kGuardBlock],
                        v3 = src[i + 3 * kGuardBlock];
            d[i] = v0;
            d[i + kGuardBlock] = v1;
            d[i + 2 * kGuardBlock] = v2;
            d[i + 3 * kGuardBlock] = v3;
        }
        for (; i < hi; i += kGuardBlock) d[i] = src[i];
    }
}

// The same check for operands that are not 16-B aligned (the flat buffers are 256-B aligned, so
// only the stateless ABI reaches it): one thread per chunk compares its sampled word bytewise and
// copies its chunk when it differs.
__global__ __launch_bounds__(kGuardWave) void k_guard_publish_bytes(const char *__restrict__ flat,
                                                                    char *__restrict__ payload, int64_t nbytes,
                                                                    int32_t *__restrict__ dirty,
                                                                    uint32_t *__restrict__ hits, int32_t gen)
{
    const int64_t n16 = nbytes >> 4;
    const int64_t samples = n16 < kGuardSamples ? n16 : kGuardSamples;
    const int64_t k = (int64_t)blockIdx.x * kGuardWave + threadIdx.x;
    int diff = 0;
    if (k < samples) {
        const int64_t o = guard_offset(k, samples, n16, (uint32_t)gen);
        for (int j = 0; j < 16; ++j) diff |= flat[o + j] != payload[o + j];
        if (k == 0)
            for (int j = 0; j < 16; ++j) diff |= flat[j] != payload[j];
        if (diff) {
            const int64_t lo = (k >= samples - 1 ? (samples > 1 ? n16 - 1 : 0) : guard_base(k, samples, n16)) << 4;
            const int64_t hi = (k >= samples - 1 ? n16 : guard_base(k + 1, samples, n16)) << 4;
            for (int64_t i = lo; i < hi; ++i) payload[i] = flat[i];
        }
    }
    if (blockIdx.x == 0 && threadIdx.x < (nbytes & 15)) {
        const int64_t j = (n16 << 4) + threadIdx.x;
        if (flat[j] != payload[j]) {
            payload[j] = flat[j];
            diff = 1;
        }
    }
    diff = __syncthreads_or(diff);
    if (diff && threadIdx.x == 0) {
        const int32_t old = atomicExch(dirty, gen);
        if (old != gen) atomicAdd(hits, 1u);
    }
}

hipError_t launch_guard_payload(char *payload, const void *flat, int64_t nbytes, int32_t *dirty, uint32_t *hits,
                                int32_t gen, hipStream_t s)
{
    if (nbytes <= 0) return hipSuccess;
    const char *src = (const char *)flat;
    const int64_t n16 = nbytes >> 4;
    const int64_t samples = n16 < kGuardSamples ? n16 : kGuardSamples;
    if (aligned16(flat) && aligned16(payload)) {
        const uint32_t g = (uint32_t)std::max<int64_t>(1, (samples + kGuardChunksPerBlock - 1) / kGuardChunksPerBlock);
        hipLaunchKernelGGL(k_guard_publish, dim3(g), dim3(kGuardBlock), 0, s, src, payload, nbytes, dirty, hits, gen);
    } else {
        const uint32_t g = (uint32_t)std::max<int64_t>(1, (samples + kGuardWave - 1) / kGuardWave);
        hipLaunchKernelGGL(k_guard_publish_bytes, dim3(g), dim3(kGuardWave), 0, s, src, payload, nbytes, dirty, hits,
                           gen);
    }
    return hipGetLastError();
}

// Window guard of resident parameters.  Between update_send and update_wait the resident
// parameters ARE the snapshot peers read; writes through `param.data` there move no version
// counter.  One launch per publish: the payload published last time -- untouched since its
// window closed, until the average after this publish overwrites that slot -- is compared with the
// samples saved when it was published (k_guard_publish's offsets of that publish's generation
// `gen`), then the samples of the payload published now (generation `cur_gen`, the offsets moved on
// by one) are saved in their place.  Each lane owns one sample, so the compare and the save of a
// sample are in one lane, in order.  `old` NULL: save only; `cur` NULL: compare only.  Layout of
// `sample`: kGuardSamples words, the tail bytes, the first word, the last word.
static_assert(kWindowSampleBytes == (kGuardSamples + 3) * 16, "window sample layout");

__global__ __launch_bounds__(kGuardWave) void k_window_roll(const char *__restrict__ old, const char *__restrict__ cur,
                                                            int64_t nbytes, char *__restrict__ sample,
                                                            int32_t *__restrict__ dirty, uint32_t *__restrict__ hits,
                                                            uint32_t *__restrict__ host, int32_t gen, int32_t cur_gen)
{
    const int64_t n16 = nbytes >> 4;
    const int64_t samples = n16 < kGuardSamples ? n16 : kGuardSamples;
    const int64_t k = (int64_t)blockIdx.x * kGuardWave + threadIdx.x;
    const bool tail = blockIdx.x == 0 && threadIdx.x < (nbytes & 15);
    char *const tail_sample = sample + kGuardSamples * 16 + threadIdx.x;
    u32x4 *const sk = reinterpret_cast<u32x4 *>(sample) + k;
    // lanes 0 and 1 of workgroup 0 also own the first and the last word (fixed, every window)
    const bool edge = blockIdx.x == 0 && threadIdx.x < 2 && n16 > 0;
    const int64_t edge_off = threadIdx.x ? (n16 - 1) << 4 : 0;
    u32x4 *const se = reinterpret_cast<u32x4 *>(sample) + kGuardSamples + 1 + threadIdx.x;
    int diff = 0;
    if (old) {
        if (k < samples) {
            const u32x4 a = *reinterpret_cast<const u32x4 *>(old + guard_offset(k, samples, n16, (uint32_t)gen));
            const u32x4 b = *sk;
            diff = (a.x != b.x) | (a.y != b.y) | (a.z != b.z) | (a.w != b.w);
        }
        if (tail) diff |= old[(n16 << 4) + threadIdx.x] != *tail_sample;
        if (edge) {
            const u32x4 a = *reinterpret_cast<const u32x4 *>(old + edge_off);
            const u32x4 b = *se;
            diff |= (a.x != b.x) | (a.y != b.y) | (a.z != b.z) | (a.w != b.w);
        }
    }
    if (cur) {
        if (k < samples) *sk = *reinterpret_cast<const u32x4 *>(cur + guard_offset(k, samples, n16, (uint32_t)cur_gen));
        if (tail) *tail_sample = cur[(n16 << 4) + threadIdx.x];
        if (edge) *se = *reinterpret_cast<const u32x4 *>(cur + edge_off);
    }
    if (!old) return;
    diff = __syncthreads_or(diff);
    if (diff && threadIdx.x == 0) {
        const int32_t prev = atomicExch(dirty, gen);
        if (prev != gen) *host = atomicAdd(hits, 1u) + 1u;   // one workgroup per window
    }
}

hipError_t launch_window_roll(const char *old, const char *cur, int64_t nbytes, char *sample, int32_t *dirty,
                              uint32_t *hits, uint32_t *host, int32_t gen, int32_t cur_gen, hipStream_t s)
{
    if (nbytes <= 0 || (!old && !cur)) return hipSuccess;
    if (!aligned16(old) || !aligned16(cur) || !aligned16(sample)) return hipErrorInvalidValue;
    const int64_t n16 = nbytes >> 4;
    const int64_t samples = n16 < kGuardSamples ? n16 : kGuardSamples;
    const uint32_t g = (uint32_t)((samples + kGuardWave - 1) / kGuardWave + (samples == 0 ? 1 : 0));
    hipLaunchKernelGGL(k_window_roll, dim3(g), dim3(kGuardWave), 0, s, old, cur, nbytes, sample, dirty, hits, host,
                       gen, cur_gen);
    return hipGetLastError();
}

// The access mix of an averaging kernel with nothing else in it, for measurement only
// (dpwa_stream_mix, bench.py `roofline.mix_ceiling`): each one-wave workgroup loads the same
// 1-KiB span of NR source buffers and stores one combination of them into the span of NW
// destinations, with exactly the product kernel's instruction shapes and cache policy
// (16-B buffer loads `nt`; the first destination stored as the parameters are, the others as the
// snapshot is) but no factor and no arithmetic beyond one add per word: the ceiling that launch
// shape reaches on this chip at a given size, timed in the same run as the product kernel.
template <int NR, int NW>
__global__ __launch_bounds__(kStreamBlock) void k_stream_mix(StreamMixArgs a)
{
    constexpr int SPAN = kStreamBlock * 16;
    const int64_t span_off = (int64_t)blockIdx.x * SPAN;
    const int lane_off = threadIdx.x * 16;
    u32x4 v[NR];
#pragma unroll
    for (int i = 0; i < NR; ++i)
        v[i] = __builtin_amdgcn_raw_buffer_load_b128(span_rsrc<SPAN>(a.src[i], span_off, a.nbytes), lane_off, 0,
                                                     kAuxStream);
    u32x4 r = v[0];
#pragma unroll
    for (int i = 1; i < NR; ++i) r = r + v[i];
    __builtin_amdgcn_raw_buffer_store_b128(r, span_rsrc<SPAN>(a.dst[0], span_off, a.nbytes), lane_off, 0,
                                           LerpPolicy<kProductPolicy>::store);
    if (NW > 1)
        __builtin_amdgcn_raw_buffer_store_b128(r, span_rsrc<SPAN>(a.dst[1], span_off, a.nbytes), lane_off, 0,
                                               LerpPolicy<kProductPolicy>::snap_store);
}

hipError_t launch_stream_mix(const StreamMixArgs &a, hipStream_t s, const LaunchTiming *timing)
{
    if (a.nr < 1 || a.nr > 2 || a.nw < 1 || a.nw > 2 || a.nbytes < 0 || (a.nbytes & 15)) return hipErrorInvalidValue;
    const uint32_t g = (uint32_t)(a.nbytes / (kStreamBlock * 16) + 1);
    void (*k)(StreamMixArgs) = a.nr == 1 ? (a.nw == 1 ? k_stream_mix<1, 1> : k_stream_mix<1, 2>)
                                         : (a.nw == 1 ? k_stream_mix<2, 1> : k_stream_mix<2, 2>);
    if (timing)
        hipExtLaunchKernelGGL(k, dim3(g), dim3(kStreamBlock), 0, s, timing->start, timing->stop, 0, a);
    else
        hipLaunchKernelGGL(k, dim3(g), dim3(kStreamBlock), 0, s, a);
    return hipGetLastError();
}

// One 64-bit word into (host-mapped) memory after everything before it on the stream: a
// system-scope release store, so the bytes written before it are visible first.  Used by
// the gossip board (board.cpp) for versions and read marks.
__global__ void k_store_u64(uint64_t *p, uint64_t v)
{
    if (threadIdx.x == 0) __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

hipError_t launch_store_u64(uint64_t *p, uint64_t v, hipStream_t s)
{
    hipLaunchKernelGGL(k_store_u64, dim3(1), dim3(64), 0, s, p, v);
    return hipGetLastError();
}

}  // namespace dpwa
