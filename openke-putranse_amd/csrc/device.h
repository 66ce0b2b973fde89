// Device-side building blocks shared by the HIP kernels (kernels.hip, universe.hip): lane-group row
// vectors with DPP reductions, the reference sampler restated per draw, and the fused per-positive
// forward/backward (group_step). See kernels.hip for the layout notes.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "graph.h"
#include "kernels.h"
#include "rng.h"

namespace pt {
namespace dev {
constexpr float kEps = 1e-12f;   // F.normalize eps

// ---------------------------------------------------------------- lane-group vectors -----------
// All-reduce sum over an aligned group of G lanes, entirely on the VALU: DPP within 16-lane rows
// (quad_perm xor1, xor2, row_half_mirror, row_mirror), then v_permlane16_swap / v_permlane32_swap
// across rows (gfx950). Every lane of the group ends with the same value (each step adds a value and
// its partner's, a commutative pair), which keeps group-uniform branches uniform.
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
template <int G>
__device__ __forceinline__ float gsum(float v) {
    if constexpr (G >= 2) v += dpp_f<0xB1>(v);    // quad_perm [1,0,3,2]
    if constexpr (G >= 4) v += dpp_f<0x4E>(v);    // quad_perm [2,3,0,1]
    if constexpr (G >= 8) v += dpp_f<0x141>(v);   // row_half_mirror
    if constexpr (G >= 16) v += dpp_f<0x140>(v);  // row_mirror
    if constexpr (G >= 32) {
        const unsigned x = __float_as_uint(v);
        const auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
        v = __uint_as_float(r[0]) + __uint_as_float(r[1]);
    }
    if constexpr (G >= 64) {
        const unsigned x = __float_as_uint(v);
        const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
        v = __uint_as_float(r[0]) + __uint_as_float(r[1]);
    }
    return v;
}

template <int G, int VEC, int KCH>
struct V {
    static constexpr int N = VEC * KCH;
    float x[N];
};

// TAIL = true: float4 chunks over a row whose length D need not be a multiple of 4 (and whose start need
// only be 4-byte aligned: unaligned 16-B global accesses are legal on gfx950): the chunk holding the row's
// last 1-3 floats is read / written element by element, the rest 16 B per lane
template <int G, int VEC, int KCH, bool TAIL = false>
__device__ __forceinline__ void vload(V<G, VEC, KCH> &o, const float *__restrict__ row, int D, int lane) {
#pragma unroll
    for (int k = 0; k < KCH; ++k) {
        const int c = k * G + lane;
        if ((k + 1) * G * VEC <= D || c * VEC < D) {   // first test is group-uniform (no exec masking)
            if constexpr (VEC == 4) {
                if (!TAIL || (c + 1) * 4 <= D) {
                    const float4 f = *reinterpret_cast<const float4 *>(row + c * 4);
                    o.x[k * 4 + 0] = f.x; o.x[k * 4 + 1] = f.y; o.x[k * 4 + 2] = f.z; o.x[k * 4 + 3] = f.w;
                } else {
#pragma unroll
                    for (int q = 0; q < 4; ++q) o.x[k * 4 + q] = c * 4 + q < D ? row[c * 4 + q] : 0.f;
                }
            } else {
#pragma unroll
                for (int q = 0; q < VEC; ++q) o.x[k * VEC + q] = row[c * VEC + q];
            }
        } else {
#pragma unroll
            for (int q = 0; q < VEC; ++q) o.x[k * VEC + q] = 0.f;
        }
    }
}

template <int G, int VEC, int KCH, bool TAIL = false>
__device__ __forceinline__ void vstore(const V<G, VEC, KCH> &o, float *__restrict__ row, int D, int lane) {
#pragma unroll
    for (int k = 0; k < KCH; ++k) {
        const int c = k * G + lane;
        if ((k + 1) * G * VEC <= D || c * VEC < D) {
            if constexpr (VEC == 4) {
                if (!TAIL || (c + 1) * 4 <= D) {
                    *reinterpret_cast<float4 *>(row + c * 4) =
                        make_float4(o.x[k * 4 + 0], o.x[k * 4 + 1], o.x[k * 4 + 2], o.x[k * 4 + 3]);
                } else {
#pragma unroll
                    for (int q = 0; q < 4; ++q)
                        if (c * 4 + q < D) row[c * 4 + q] = o.x[k * 4 + q];
                }
            } else {
#pragma unroll
                for (int q = 0; q < VEC; ++q) row[c * VEC + q] = o.x[k * VEC + q];
            }
        }
    }
}

template <int G, int VEC, int KCH, bool TAIL = false>
__device__ __forceinline__ void vatomic(const V<G, VEC, KCH> &o, float *__restrict__ row, int D, int lane) {
#pragma unroll
    for (int k = 0; k < KCH; ++k) {
        const int c = k * G + lane;
        if (c * VEC < D) {
#pragma unroll
            for (int q = 0; q < VEC; ++q)
                if (!TAIL || c * VEC + q < D) atomicAdd(row + c * VEC + q, o.x[k * VEC + q]);
        }
    }
}

// Address-space-typed pointers: rows reached through pointers loaded from memory (a universe descriptor)
// or selected at run time between LDS and HBM are generic ("flat") to the compiler, and a flat access
// counts in BOTH vmcnt and lgkmcnt - every LDS wait then also waits for the in-flight HBM loads. Kernels
// that know where a row lives cast once to these types, so each access is a global_* or ds_* instruction.
typedef __attribute__((address_space(1))) float gfloat;
typedef __attribute__((address_space(3))) float lfloat;
typedef __attribute__((address_space(1))) int32_t gint32;
typedef __attribute__((address_space(3))) int32_t lint32;
typedef __attribute__((address_space(3))) int lint;
typedef __attribute__((address_space(3))) uint64_t luint64;
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) f32x4 gf32x4;
typedef __attribute__((address_space(3))) f32x4 lf32x4;
typedef __attribute__((address_space(1))) i32x4 gi32x4;

template <typename FP, typename F4P, int G, int VEC, int KCH>
__device__ __forceinline__ void vload_t(V<G, VEC, KCH> &o, FP row, int D, int lane) {
#pragma unroll
    for (int k = 0; k < KCH; ++k) {
        const int c = k * G + lane;
        if ((k + 1) * G * VEC <= D || c * VEC < D) {
            if constexpr (VEC == 4) {
                const f32x4 f = *reinterpret_cast<F4P>(row + c * 4);
                o.x[k * 4 + 0] = f.x; o.x[k * 4 + 1] = f.y; o.x[k * 4 + 2] = f.z; o.x[k * 4 + 3] = f.w;
            } else {
#pragma unroll
                for (int q = 0; q < VEC; ++q) o.x[k * VEC + q] = row[c * VEC + q];
            }
        } else {
#pragma unroll
            for (int q = 0; q < VEC; ++q) o.x[k * VEC + q] = 0.f;
        }
    }
}
template <typename FP, typename F4P, int G, int VEC, int KCH>
__device__ __forceinline__ void vstore_t(const V<G, VEC, KCH> &o, FP row, int D, int lane) {
#pragma unroll
    for (int k = 0; k < KCH; ++k) {
        const int c = k * G + lane;
        if ((k + 1) * G * VEC <= D || c * VEC < D) {
            if constexpr (VEC == 4) {
                const f32x4 f = {o.x[k * 4 + 0], o.x[k * 4 + 1], o.x[k * 4 + 2], o.x[k * 4 + 3]};
                *reinterpret_cast<F4P>(row + c * 4) = f;
            } else {
#pragma unroll
                for (int q = 0; q < VEC; ++q) row[c * VEC + q] = o.x[k * VEC + q];
            }
        }
    }
}
template <int G, int VEC, int KCH>
__device__ __forceinline__ void vload(V<G, VEC, KCH> &o, const gfloat *row, int D, int lane) {
    vload_t<const gfloat *, const gf32x4 *>(o, row, D, lane);
}
template <int G, int VEC, int KCH>
__device__ __forceinline__ void vload(V<G, VEC, KCH> &o, const lfloat *row, int D, int lane) {
    vload_t<const lfloat *, const lf32x4 *>(o, row, D, lane);
}
template <int G, int VEC, int KCH>
__device__ __forceinline__ void vstore(const V<G, VEC, KCH> &o, gfloat *row, int D, int lane) {
    vstore_t<gfloat *, gf32x4 *>(o, row, D, lane);
}
template <int G, int VEC, int KCH>
__device__ __forceinline__ void vstore(const V<G, VEC, KCH> &o, lfloat *row, int D, int lane) {
    vstore_t<lfloat *, lf32x4 *>(o, row, D, lane);
}
// float atomic adds into an LDS row (ds_add_f32) / an HBM row (global_atomic_add_f32)
template <int G, int VEC, int KCH>
__device__ __forceinline__ void vatomic(const V<G, VEC, KCH> &o, lfloat *row, int D, int lane) {
#pragma unroll
    for (int k = 0; k < KCH; ++k) {
        const int c = k * G + lane;
        if (c * VEC < D) {
#pragma unroll
            for (int q = 0; q < VEC; ++q)
                __hip_atomic_fetch_add(row + c * VEC + q, o.x[k * VEC + q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    }
}
template <int G, int VEC, int KCH>
__device__ __forceinline__ void vatomic(const V<G, VEC, KCH> &o, gfloat *row, int D, int lane) {
#pragma unroll
    for (int k = 0; k < KCH; ++k) {
        const int c = k * G + lane;
        if (c * VEC < D) {
#pragma unroll
            for (int q = 0; q < VEC; ++q)
                __hip_atomic_fetch_add(row + c * VEC + q, o.x[k * VEC + q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

template <int G, int VEC, int KCH>
__device__ __forceinline__ float vdot(const V<G, VEC, KCH> &a, const V<G, VEC, KCH> &b) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < V<G, VEC, KCH>::N; ++i) s += a.x[i] * b.x[i];
    return gsum<G>(s);
}

template <int G, int VEC, int KCH>
__device__ __forceinline__ void vzero(V<G, VEC, KCH> &a) {
#pragma unroll
    for (int i = 0; i < V<G, VEC, KCH>::N; ++i) a.x[i] = 0.f;
}

template <int G, int VEC, int KCH>
__device__ __forceinline__ bool vnonzero(const V<G, VEC, KCH> &a) {
    int nz = 0;
#pragma unroll
    for (int i = 0; i < V<G, VEC, KCH>::N; ++i) nz |= a.x[i] != 0.f;
    return gsum<G>((float)nz) != 0.f;
}

// Raw-buffer row access (buffer_load / buffer_store with a table-wide resource): lanes past the row
// end get an out-of-range offset, so the hardware returns 0 / drops the store - no exec masking and
// no branches around the access, which keeps s_waitcnt counting exact for software pipelining.
// Callers check that every byte offset fits in 31 bits.
typedef unsigned int pt_u32x4 __attribute__((ext_vector_type(4)));
constexpr uint32_t kOob = 0x80000000u;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void *base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), 0, (int)bytes, 0x00020000);
}
// AUX: the buffer instruction's cache-policy bits (16 = sc1: agent-coherent, past the CU's L1 - the hand-off form of
// MI355X_MICROARCH.md for data another workgroup wrote or reads)
template <int G, int VEC, int KCH, int AUX = 0>
__device__ __forceinline__ void bload(V<G, VEC, KCH> &o, __amdgpu_buffer_rsrc_t rs, uint32_t row_bytes, int D,
                                      int lane) {
#pragma unroll
    for (int k = 0; k < KCH; ++k) {
        const int c = k * G + lane;
        const uint32_t off = c * VEC < D ? row_bytes + (uint32_t)(c * VEC * 4) : kOob;
        if constexpr (VEC == 4) {
            const pt_u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, AUX);
            o.x[k * 4 + 0] = __uint_as_float(v.x); o.x[k * 4 + 1] = __uint_as_float(v.y);
            o.x[k * 4 + 2] = __uint_as_float(v.z); o.x[k * 4 + 3] = __uint_as_float(v.w);
        } else {
            static_assert(VEC == 1, "bload: VEC 1 or 4");
            o.x[k] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, AUX));
        }
    }
}
template <int G, int VEC, int KCH, int AUX = 0>
__device__ __forceinline__ void bstore(const V<G, VEC, KCH> &o, __amdgpu_buffer_rsrc_t rs, uint32_t row_bytes, int D,
                                       int lane) {
#pragma unroll
    for (int k = 0; k < KCH; ++k) {
        const int c = k * G + lane;
        const uint32_t off = c * VEC < D ? row_bytes + (uint32_t)(c * VEC * 4) : kOob;
        if constexpr (VEC == 4) {
            const pt_u32x4 v = {__float_as_uint(o.x[k * 4 + 0]), __float_as_uint(o.x[k * 4 + 1]),
                                __float_as_uint(o.x[k * 4 + 2]), __float_as_uint(o.x[k * 4 + 3])};
            __builtin_amdgcn_raw_buffer_store_b128(v, rs, off, 0, AUX);
        } else {
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(o.x[k]), rs, off, 0, AUX);
        }
    }
}

// sqrt / reciprocal: correctly rounded by default; FAST = the hardware v_sqrt_f32 / v_rcp_f32 (1 ulp),
// used by the training step, whose results are compared with a tolerance anyway (the scoring kernels
// that feed ranking keep the IEEE forms)
template <bool FAST>
__device__ __forceinline__ float fsqrt(float x) {
    if constexpr (FAST) return __builtin_amdgcn_sqrtf(x); else return sqrtf(x);
}
template <bool FAST>
__device__ __forceinline__ float frcp(float x) {
    if constexpr (FAST) return __builtin_amdgcn_rcpf(x); else return 1.0f / x;
}

// group-uniform value -> scalar register when the group is the whole wave (branches on it become
// scalar branches, addresses built from it scalar)
template <int G>
__device__ __forceinline__ int32_t uni(int32_t x) {
    if constexpr (G == 64) return __builtin_amdgcn_readfirstlane(x); else return x;
}
template <int G>
__device__ __forceinline__ float uni(float x) {
    if constexpr (G == 64) return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(x))); else return x;
}

// F.normalize(x, 2, -1): out = x / max(||x||, eps); returns ||x||
template <bool FAST = false, int G, int VEC, int KCH>
__device__ __forceinline__ float vnormalize(const V<G, VEC, KCH> &x, V<G, VEC, KCH> &out) {
    const float n = fsqrt<FAST>(vdot(x, x));
    const float inv = frcp<FAST>(n > kEps ? n : kEps);   // one division per row, then multiplies
#pragma unroll
    for (int i = 0; i < V<G, VEC, KCH>::N; ++i) out.x[i] = x.x[i] * inv;
    return n;
}

// backward of F.normalize at raw x with norm n: (g - x (x.g)/n^2) / n   (clamp_min branch: g / eps)
template <bool FAST = false, int G, int VEC, int KCH>
__device__ __forceinline__ void vnormalize_bwd(const V<G, VEC, KCH> &x, float n, const V<G, VEC, KCH> &g,
                                               V<G, VEC, KCH> &out) {
    if (n > kEps) {
        const float inv = frcp<FAST>(n);
        const float c = vdot(g, x) * (inv * inv);
#pragma unroll
        for (int i = 0; i < V<G, VEC, KCH>::N; ++i) out.x[i] = (g.x[i] - x.x[i] * c) * inv;
    } else {
#pragma unroll
        for (int i = 0; i < V<G, VEC, KCH>::N; ++i) out.x[i] = g.x[i] / kEps;
    }
}

// ||v||_p for p in {1,2}
template <bool FAST = false, int G, int VEC, int KCH>
__device__ __forceinline__ float vpnorm(const V<G, VEC, KCH> &v, int p) {
    float s = 0.f;
    if (p == 1) {
#pragma unroll
        for (int i = 0; i < V<G, VEC, KCH>::N; ++i) s += fabsf(v.x[i]);
        return gsum<G>(s);
    }
#pragma unroll
    for (int i = 0; i < V<G, VEC, KCH>::N; ++i) s += v.x[i] * v.x[i];
    return fsqrt<FAST>(gsum<G>(s));
}

// ds * d||v||_p/dv : p=1 sgn(v)*ds (sgn 0 = 0), p=2 v*(ds/||v||) masked at ||v|| = 0
template <bool FAST = false, int G, int VEC, int KCH>
__device__ __forceinline__ void vpnorm_bwd(const V<G, VEC, KCH> &v, float nv, int p, float ds, V<G, VEC, KCH> &g) {
    if (p == 1) {
#pragma unroll
        for (int i = 0; i < V<G, VEC, KCH>::N; ++i) g.x[i] = v.x[i] > 0.f ? ds : (v.x[i] < 0.f ? -ds : 0.f);
    } else {
        const float k = nv == 0.f ? 0.f : (FAST ? ds * frcp<true>(nv) : ds / nv);
#pragma unroll
        for (int i = 0; i < V<G, VEC, KCH>::N; ++i) g.x[i] = v.x[i] * k;
    }
}

// ---------------------------------------------------------------- sampler --------------------
__device__ __forceinline__ int64_t rand_max(uint64_t &s, int64_t x) { return (int64_t)(lcg_next(s) % (uint64_t)x); }

// Boundary search of the filtered corruption (Corrupt.h:43-55). The reference bisects for the largest m
// in its open interval with f(m) = vals[m] - m + lo - 1 < tmp. vals (the known partners of a run) is
// strictly increasing, so f is nondecreasing and that boundary is unique: any probe order that keeps
// f(l) < tmp <= f(r) ends at the same l. Probes interpolate between (l, f(l)) and (r, f(r)) - the
// entity ids of a run are spread over [0, E), so long runs take ~log log n dependent loads instead of
// log n - with a bisection step after any step that did not halve the interval (at most 2 log n).
struct RunSearch {
    const int32_t *vals;
    int32_t lo, l, r, fl, fr, tmp;
    bool bis;
};

// closed run [lo, hi] with f(lo) < tmp <= f(hi) (the reference's two early exits already failed)
__device__ __forceinline__ RunSearch run_search(const int32_t *vals, int32_t lo, int32_t hi, int32_t vlo, int32_t vhi,
                                                int32_t tmp) {
    return RunSearch{vals, lo, lo, hi, vlo - 1, vhi - hi + lo - 1, tmp, false};
}
__device__ __forceinline__ bool rs_open(const RunSearch &q) { return q.l + 1 < q.r; }
__device__ __forceinline__ int32_t rs_probe(const RunSearch &q) {
    if (q.bis) return (q.l + q.r) >> 1;
    const float frac = __fdividef((float)(q.tmp - q.fl), (float)(q.fr - q.fl));
    const int32_t m = q.l + (int32_t)(frac * (float)(q.r - q.l));
    return m <= q.l ? q.l + 1 : (m >= q.r ? q.r - 1 : m);
}
__device__ __forceinline__ void rs_update(RunSearch &q, int32_t m, int32_t v) {
    const int32_t f = v - m + q.lo - 1, width = q.r - q.l;
    if (f < q.tmp) { q.l = m; q.fl = f; } else { q.r = m; q.fr = f; }
    q.bis = 2 * (q.r - q.l) > width;
}
// the corrupted entity once the search is closed
__device__ __forceinline__ int64_t rs_entity(const RunSearch &q) { return (int64_t)q.tmp + q.l - q.lo + 1; }

// Filtered corruption (Corrupt.h:27-56 / :75-104): `vals` is the searched column of the sorted list
// (trainHead[].t for corrupt_head, trainTail[].h for corrupt_tail) and [lo, hi] the run of known
// partners of the positive's (entity, relation) - the [ll, rr] of the reference's two binary searches,
// precomputed per triple (TripleRec). The draw, the early exits and the boundary are the reference's.
template <typename VP>
__device__ __forceinline__ int64_t corrupt_in_run(VP vals, int64_t lo, int64_t hi, int64_t E, uint64_t &s) {
    const int64_t tmp = rand_max(s, E - (hi - lo + 1));
    const int32_t vlo = vals[lo], vhi = vals[hi];
    if (tmp < vlo) return tmp;
    if (tmp > vhi - hi + lo - 1) return tmp + hi - lo + 1;
    RunSearch q = run_search(nullptr, (int32_t)lo, (int32_t)hi, vlo, vhi, (int32_t)tmp);   // (vals read here)
    while (rs_open(q)) {
        const int32_t m = rs_probe(q);
        rs_update(q, m, vals[m]);
    }
    return rs_entity(q);
}

// state of the sampler stream that produces positive b of call `call` after the current states
// (Base.cpp:200-207 split: thread id owns positives [id*per, min((id+1)*per, bs)) of every call)
template <typename SP>
__device__ __forceinline__ uint64_t positive_state(SP states, int64_t threads, int64_t bs, int64_t b, int64_t dpp,
                                                   int64_t call = 0) {
    const int64_t per = bs % threads == 0 ? bs / threads : bs / threads + 1;
    const int64_t id = b / per;
    int64_t len = bs - id * per;
    len = len > per ? per : len;
    return lcg_jump(states[id], (uint64_t)((call * len + (b - id * per)) * dpp));
}

struct PosDraw {
    int64_t h, r, t;
    int32_t hr_lo, hr_hi, tr_lo, tr_hi;
    uint64_t s1;   // stream state after the positive's index draw
    int64_t idx;   // trainList index of the positive
};

// The training graph as HBM-typed pointers (DeviceGraph's fields are generic: fine as kernel arguments,
// which the compiler promotes to global, but flat when loaded from a descriptor in memory)
struct DeviceGraphG {
    int64_t ent_total, rel_total, train_total;
    const gi32x4 *rec;          // TripleRec[train_total] as pairs of int4
    const gint32 *head_t, *tail_h;
    const gfloat *bern_prob;
};
__device__ __forceinline__ DeviceGraphG as_global(const DeviceGraph &g) {
    return DeviceGraphG{g.ent_total, g.rel_total, g.train_total, (const gi32x4 *)(const void *)g.rec,
                        (const gint32 *)g.head_t, (const gint32 *)g.tail_h, (const gfloat *)g.bern_prob};
}
__device__ __forceinline__ void graph_rec(const DeviceGraph &g, int64_t i, i32x4 &a, i32x4 &c) {
    const i32x4 *p = reinterpret_cast<const i32x4 *>(g.rec + i);
    a = p[0];
    c = p[1];
}
__device__ __forceinline__ void graph_rec(const DeviceGraphG &g, int64_t i, i32x4 &a, i32x4 &c) {
    a = g.rec[2 * i];
    c = g.rec[2 * i + 1];
}

// positive b: i = rand_max(trainTotal), trainList[i] (Base.cpp:210-215)
template <typename GR, typename SP>
__device__ __forceinline__ PosDraw draw_positive(const GR &g, SP states, int64_t threads, int64_t bs, int64_t b,
                                                 int64_t dpp, int64_t call = 0) {
    uint64_t s = positive_state(states, threads, bs, b, dpp, call);
    const int64_t i = rand_max(s, g.train_total);
    i32x4 a, c;
    graph_rec(g, i, a, c);
    return PosDraw{a.x, a.y, a.z, a.w, c.x, c.y, c.z, s, i};
}

// negative k of a positive (stream offsets 1+2k coin, 2+2k corruption; Base.cpp:217-232): returns the
// corrupted entity, *tail_side = 1 when the tail was replaced (corrupt_head), 0 when the head was
template <typename GR>
__device__ __forceinline__ int64_t draw_negative(const GR &g, const PosDraw &p, int64_t k, int bern, int filter,
                                                 int *tail_side) {
    uint64_t s = lcg_jump(p.s1, (uint64_t)(2 * k));
    const float prob = bern ? g.bern_prob[p.r] : 500.f;
    const int64_t E = g.ent_total;
    if ((float)(lcg_next(s) % 1000ULL) < prob) {
        *tail_side = 1;
        if (filter) return corrupt_in_run(g.head_t, p.hr_lo, p.hr_hi, E, s);
        const int64_t tmp = rand_max(s, E - 1);   // skips the passed entity h (Corrupt.h:18-25)
        return tmp < p.h ? tmp : tmp + 1;
    }
    *tail_side = 0;
    if (filter) return corrupt_in_run(g.tail_h, p.tr_lo, p.tr_hi, E, s);
    const int64_t tmp = rand_max(s, E - 1);       // skips t (Corrupt.h:68-74)
    return tmp < p.t ? tmp : tmp + 1;
}

__device__ __forceinline__ void advance_states(uint64_t *states, int64_t threads, int64_t bs, int64_t dpp, int lane) {
    if (lane < threads) {
        const int64_t per = bs % threads == 0 ? bs / threads : bs / threads + 1;
        int64_t len = bs - lane * per;
        len = len < 0 ? 0 : (len > per ? per : len);
        states[lane] = lcg_jump(states[lane], (uint64_t)(len * dpp));
    }
}

// One positive group: forward + MarginLoss + backward for the positive and its `neg` negatives.
// Gradient conventions per table (the apply pass finishes them):
//   TransE: ent and rel gradients in normalized space (the apply pass multiplies by the normalize
//           Jacobian of the pre-step row; sum-then-Jacobian == Jacobian-then-sum, it is linear);
//   TransH: ent gradients raw (their projection/normalize Jacobians depend on the relation, so they are
//           applied here), rel in normalized space, norm_vector in normalized (n-hat) space.
// Negatives are given by `get_neg(k, &h, &t, &r)`; rows equal to the positive's reuse its registers
// and accumulate on chip, other rows go straight to the sink.
template <int MODEL, int G, int VEC, int KCH, typename Sink, typename NegFn>
__device__ __forceinline__ float group_step(const StepParams &P, int64_t hp, int64_t rp, int64_t tp, int64_t neg,
                                            NegFn get_neg, const Sink &sink, int lane) {
    using Vec = V<G, VEC, KCH>;
    const int D = (int)P.dim;
    const int p = P.p_norm;
    const bool nf = P.norm_flag != 0;
    // ---- positive
    Vec H, T, Rr, W, nW, hh, th, rh, vpos;
    float hn = 0, tn = 0, hdot = 0, tdot = 0;
    vload(H, P.ent + hp * D, D, lane);
    vload(T, P.ent + tp * D, D, lane);
    vload(Rr, P.rel + rp * D, D, lane);
    Vec Hs = H, Ts = T;   // scored entity vectors (projected for TransH)
    if constexpr (MODEL == 1) {
        vload(W, P.normv + rp * D, D, lane);
        vnormalize(W, nW);
        hdot = vdot(H, nW);
        tdot = vdot(T, nW);
#pragma unroll
        for (int i = 0; i < Vec::N; ++i) {
            Hs.x[i] = H.x[i] - hdot * nW.x[i];
            Ts.x[i] = T.x[i] - tdot * nW.x[i];
        }
    }
    if (nf) {
        hn = vnormalize(Hs, hh);
        vnormalize(Rr, rh);
        tn = vnormalize(Ts, th);
    } else {
        hh = Hs; rh = Rr; th = Ts;
    }
#pragma unroll
    for (int i = 0; i < Vec::N; ++i) vpos.x[i] = (hh.x[i] + rh.x[i]) - th.x[i];
    const float ps = vpnorm(vpos, p);

    Vec aH, aT, aR, aW;   // on-chip accumulators of the positive's rows
    vzero(aH); vzero(aT); vzero(aR); vzero(aW);
    float csum = 0.f, lsum = 0.f;
    const float m = P.margin;
    const float inv = P.inv_count;

    for (int64_t k = 0; k < neg; ++k) {
        int64_t hk, tk, rk;
        get_neg(k, hk, tk, rk);
        const bool same_r = rk == rp;
        // relation row of the negative
        Vec Rk, rkh, Wk, nWk;
        if (same_r) {
            rkh = rh;
            if constexpr (MODEL == 1) { nWk = nW; Wk = W; }
        } else {
            vload(Rk, P.rel + rk * D, D, lane);
            if (nf) vnormalize(Rk, rkh); else rkh = Rk;
            if constexpr (MODEL == 1) {
                vload(Wk, P.normv + rk * D, D, lane);
                vnormalize(Wk, nWk);
            }
        }
        // entity rows of the negative: reuse the positive's when the (row, relation) matches
        Vec Ek[2], Eks[2], ekh[2];
        float ekn[2], ekdot[2];
        int role[2];   // 0: row hp, 1: row tp, -1: other
        const int64_t ids[2] = {hk, tk};
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            const int64_t e = ids[s];
            role[s] = !same_r ? -1 : (e == hp ? 0 : (e == tp ? 1 : -1));
            if (role[s] == 0) {
                Ek[s] = H; Eks[s] = Hs; ekh[s] = hh; ekn[s] = hn; ekdot[s] = hdot;
            } else if (role[s] == 1) {
                Ek[s] = T; Eks[s] = Ts; ekh[s] = th; ekn[s] = tn; ekdot[s] = tdot;
            } else {
                vload(Ek[s], P.ent + e * D, D, lane);
                Eks[s] = Ek[s];
                ekdot[s] = 0.f;
                if constexpr (MODEL == 1) {
                    ekdot[s] = vdot(Ek[s], nWk);
#pragma unroll
                    for (int i = 0; i < Vec::N; ++i) Eks[s].x[i] = Ek[s].x[i] - ekdot[s] * nWk.x[i];
                }
                if (nf) ekn[s] = vnormalize(Eks[s], ekh[s]); else { ekh[s] = Eks[s]; ekn[s] = 0.f; }
            }
        }
        Vec vk;
#pragma unroll
        for (int i = 0; i < Vec::N; ++i) vk.x[i] = (ekh[0].x[i] + rkh.x[i]) - ekh[1].x[i];
        const float ns = vpnorm(vk, p);
        const float a = ps - ns;
        lsum += a > -m ? a : -m;
        const float c = a > -m ? inv : (a == -m ? inv * 0.5f : 0.f);
        if (c == 0.f) continue;
        csum += c;
        Vec g;
        vpnorm_bwd(vk, ns, p, -c, g);   // d loss / d v_k
        // relation (normalized space)
        if (same_r) {
#pragma unroll
            for (int i = 0; i < Vec::N; ++i) aR.x[i] += g.x[i];
        } else {
            sink.rel(rk, g, D, lane);
        }
        Vec gw;   // TransH: d/d n-hat of this negative's relation
        if constexpr (MODEL == 1) vzero(gw);
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            Vec gs;   // d/d(normalized scored entity): +g for the head, -g for the tail
#pragma unroll
            for (int i = 0; i < Vec::N; ++i) gs.x[i] = s == 0 ? g.x[i] : -g.x[i];
            if (role[s] >= 0) {
                Vec &acc = role[s] == 0 ? aH : aT;
#pragma unroll
                for (int i = 0; i < Vec::N; ++i) acc.x[i] += gs.x[i];
                continue;
            }
            if constexpr (MODEL == 0) {
                sink.ent(ids[s], gs, D, lane);
            } else {
                Vec gp;   // through normalize of the projected vector
                if (nf) vnormalize_bwd(Eks[s], ekn[s], gs, gp); else gp = gs;
                const float ng = vdot(nWk, gp);
                Vec ge;
#pragma unroll
                for (int i = 0; i < Vec::N; ++i) {
                    ge.x[i] = gp.x[i] - nWk.x[i] * ng;
                    gw.x[i] -= ekdot[s] * gp.x[i] + ng * Ek[s].x[i];
                }
                sink.ent(ids[s], ge, D, lane);
            }
        }
        if constexpr (MODEL == 1) {
            if (same_r) {
#pragma unroll
                for (int i = 0; i < Vec::N; ++i) aW.x[i] += gw.x[i];
            } else if (vnonzero(gw)) {
                sink.norm(rk, gw, D, lane);
            }
        }
    }
    // ---- positive backward
    if (csum != 0.f) {
        Vec g;
        vpnorm_bwd(vpos, ps, p, csum, g);
#pragma unroll
        for (int i = 0; i < Vec::N; ++i) {
            aH.x[i] += g.x[i];
            aR.x[i] += g.x[i];
            aT.x[i] -= g.x[i];
        }
    }
    if (vnonzero(aR)) sink.rel(rp, aR, D, lane);
    if constexpr (MODEL == 0) {
        if (vnonzero(aH)) sink.ent(hp, aH, D, lane);
        if (vnonzero(aT)) sink.ent(tp, aT, D, lane);
    } else {
        // positive-row accumulators are in normalized-projected space: finish them once
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            Vec &acc = s == 0 ? aH : aT;
            if (!vnonzero(acc)) continue;
            const Vec &E = s == 0 ? H : T;
            const Vec &Es = s == 0 ? Hs : Ts;
            const float en = s == 0 ? hn : tn;
            const float edot = s == 0 ? hdot : tdot;
            Vec gp;
            if (nf) vnormalize_bwd(Es, en, acc, gp); else gp = acc;
            const float ng = vdot(nW, gp);
            Vec ge;
#pragma unroll
            for (int i = 0; i < Vec::N; ++i) {
                ge.x[i] = gp.x[i] - nW.x[i] * ng;
                aW.x[i] -= edot * gp.x[i] + ng * E.x[i];
            }
            sink.ent(s == 0 ? hp : tp, ge, D, lane);
        }
        if (vnonzero(aW)) sink.norm(rp, aW, D, lane);
    }
    return lsum;
}

}  // namespace dev
}  // namespace pt
