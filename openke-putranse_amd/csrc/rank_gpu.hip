// Link-prediction ranks straight from global-order score rows (PuTransE global energy estimation).
//
// The reference builds, per test query, a candidate-order score vector [truth, 0..E-1 \ truth]
// (global_energy_estimation, Parallel_Universe_Config.py:556-601) and ranks it on the CPU
// (testHead/testTail, Test.h:118-359; validHead/validTail, Valid.h:117-240):
//   raw  = #{j >= 1 : con[j] < con[0]}
//   filt = raw minus the candidates j whose triple is known (_find over tripleList, Corrupt.h:188-199)
//   con[0] == inf:  raw = E, filt = E - #{known candidates}.
// Candidate order does not change these counts, so here a query is ranked directly on its key's
// global-order row val(e) (after the null_vector replacement of +inf entries, :590-599):
//   raw  = #{e != truth : val(e) < val(truth)}
//   filt = raw - #{p in partners(anchor, r), p != truth : val(p) < val(truth)}
// with partners(anchor, r) the known entities completing the query's (anchor, r) (host CSR,
// pt_known_partners). One workgroup per query streams the E floats of its row (coalesced) and its
// partner list; HBM-bound, 4 B per (query, candidate).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "kernels.h"

namespace pt {
namespace dev {

__device__ __forceinline__ float repl_val(float v, float repl) { return v == INFINITY ? repl : v; }

__global__ __launch_bounds__(256) void k_rank_rows(const float *__restrict__ rows, int64_t E,
                                                   const int64_t *__restrict__ row_of, const int64_t *__restrict__ truth,
                                                   const float *__restrict__ repl, const int64_t *__restrict__ part_off,
                                                   const int64_t *__restrict__ part, int64_t *__restrict__ raw,
                                                   int64_t *__restrict__ filt) {
    __shared__ int64_t red[2][4];
    const int64_t q = blockIdx.x;
    const float *row = rows + row_of[q] * E;
    const float rp = repl ? repl[q] : INFINITY;
    const int64_t tr = truth[q];
    const float s0 = repl_val(row[tr], rp);
    const bool inf0 = s0 == INFINITY;
    int64_t below = 0, known_below = 0;
    if (!inf0) {
        // vectorised stream of the row (16-B loads where aligned)
        const int64_t head = (4 - (((uintptr_t)row >> 2) & 3)) & 3;
        for (int64_t e = threadIdx.x; e < head && e < E; e += blockDim.x) below += repl_val(row[e], rp) < s0;
        const int64_t n4 = (E - head) / 4;
        const float4 *r4 = reinterpret_cast<const float4 *>(row + head);
        for (int64_t i = threadIdx.x; i < n4; i += blockDim.x) {
            const float4 v = r4[i];
            below += (repl_val(v.x, rp) < s0) + (repl_val(v.y, rp) < s0) + (repl_val(v.z, rp) < s0) +
                     (repl_val(v.w, rp) < s0);
        }
        for (int64_t e = head + 4 * n4 + threadIdx.x; e < E; e += blockDim.x) below += repl_val(row[e], rp) < s0;
    }
    for (int64_t k = part_off[q] + threadIdx.x; k < part_off[q + 1]; k += blockDim.x) {
        const int64_t p = part[k];
        if (p == tr) continue;
        known_below += inf0 ? 1 : (repl_val(row[p], rp) < s0);
    }
    // workgroup reduction: wave shuffles then LDS
    for (int o = 32; o > 0; o >>= 1) {
        below += __shfl_down(below, o, 64);
        known_below += __shfl_down(known_below, o, 64);
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        red[0][w] = below;
        red[1][w] = known_below;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        int64_t b = 0, kb = 0;
        for (int i = 0; i < (int)(blockDim.x >> 6); ++i) {
            b += red[0][i];
            kb += red[1][i];
        }
        if (inf0) {
            raw[q] = E;
            filt[q] = E - kb;
        } else {
            raw[q] = b;
            filt[q] = b - kb;
        }
    }
}

// Type-constrained counts (testHead/testTail with type_constrain, Test.h:127-130, :168-178, :288-298).
// The reference walks candidate POSITIONS j = 1..E-1 and matches j against the relation's sorted type
// list as an ENTITY id: for type entity j it compares con[j], the score of the candidate at position j
// - entity j-1 when j-1 < truth, else entity j - and its filter asks _find about entity j itself.
// Restated on the global-order row: one workgroup per query walks the relation's type list (duplicates
// and ids outside [1, E) skipped, as the reference's merge skips them), gathers val(c(j)) and bisects
// the query's ascending partner list for j. Nothing is counted when the truth's score is +inf.
__global__ __launch_bounds__(256) void k_rank_types(const float *__restrict__ rows, int64_t E,
                                                    const int64_t *__restrict__ row_of, const int64_t *__restrict__ truth,
                                                    const float *__restrict__ repl, const int64_t *__restrict__ rel,
                                                    const int64_t *__restrict__ type_lef,
                                                    const int64_t *__restrict__ type_rig,
                                                    const int64_t *__restrict__ types, const int64_t *__restrict__ part_off,
                                                    const int64_t *__restrict__ part, int64_t *__restrict__ raw,
                                                    int64_t *__restrict__ filt) {
    __shared__ int64_t red[2][4];
    const int64_t q = blockIdx.x;
    const float *row = rows + row_of[q] * E;
    const float rp = repl ? repl[q] : INFINITY;
    const int64_t tr = truth[q];
    const float s0 = repl_val(row[tr], rp);
    int64_t below = 0, unknown_below = 0;
    if (s0 != INFINITY) {
        const int64_t r = rel[q], lo = type_lef[r], hi = type_rig[r];
        const int64_t plo = part_off[q], phi = part_off[q + 1];
        for (int64_t k = lo + threadIdx.x; k < hi; k += blockDim.x) {
            const int64_t j = types[k];
            if (j < 1 || j >= E || (k > lo && types[k - 1] == j)) continue;
            const int64_t c = j - 1 < tr ? j - 1 : j;
            if (!(repl_val(row[c], rp) < s0)) continue;
            ++below;
            int64_t a = plo, b = phi;   // first partner >= j
            while (a < b) {
                const int64_t m = (a + b) >> 1;
                if (part[m] < j) a = m + 1; else b = m;
            }
            unknown_below += !(a < phi && part[a] == j);
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        below += __shfl_down(below, o, 64);
        unknown_below += __shfl_down(unknown_below, o, 64);
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        red[0][w] = below;
        red[1][w] = unknown_below;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        int64_t b = 0, u = 0;
        for (int i = 0; i < (int)(blockDim.x >> 6); ++i) {
            b += red[0][i];
            u += red[1][i];
        }
        raw[q] = b;
        filt[q] = u;
    }
}

}  // namespace dev

hipError_t launch_rank_types(const float *rows, int64_t E, const int64_t *row_of, const int64_t *truth,
                             const float *repl, const int64_t *rel, const int64_t *type_lef, const int64_t *type_rig,
                             const int64_t *types, const int64_t *part_off, const int64_t *part, int64_t nq,
                             int64_t *raw, int64_t *filt, hipStream_t st) {
    if (nq <= 0) return hipSuccess;
    for (int64_t off = 0; off < nq; off += 1 << 30) {
        const int64_t n = nq - off < (1 << 30) ? nq - off : (1 << 30);
        hipLaunchKernelGGL(dev::k_rank_types, dim3((unsigned)n), dim3(256), 0, st, rows, E, row_of + off, truth + off,
                           repl ? repl + off : nullptr, rel + off, type_lef, type_rig, types, part_off + off, part,
                           raw + off, filt + off);
    }
    return hipGetLastError();
}

hipError_t launch_rank_rows(const float *rows, int64_t E, const int64_t *row_of, const int64_t *truth,
                            const float *repl, const int64_t *part_off, const int64_t *part, int64_t nq, int64_t *raw,
                            int64_t *filt, hipStream_t st) {
    if (nq <= 0) return hipSuccess;
    for (int64_t off = 0; off < nq; off += 1 << 30) {
        const int64_t n = nq - off < (1 << 30) ? nq - off : (1 << 30);
        hipLaunchKernelGGL(dev::k_rank_rows, dim3((unsigned)n), dim3(256), 0, st, rows, E, row_of + off, truth + off,
                           repl ? repl + off : nullptr, part_off + off, part, raw + off, filt + off);
    }
    return hipGetLastError();
}

}  // namespace pt
