// Initial tables of a universe's model drawn on the GPU, bit-identical to the torch CPU generator's.
//
// The reference builds every universe's model on the CPU after torch.manual_seed(seed0 + k)
// (Parallel_Universe_Config.py:157-161, 169-177): nn.Embedding draws N(0, 1) into each table (normal_), then
// TransE / TransH overwrite them with xavier_uniform_ (TransE.py:17-36, TransH.py:17-42). Only the uniform draws
// survive; the normal_ calls matter through the generator draws they consume (the host counts them,
// Model._normal_draws). torch's CPU generator is MT19937 seeded by init_genrand(seed mod 2^32); a float
// uniform_(from, to) consumes one 32-bit output x per element and stores
//     (float)((double)(x & (2^24 - 1)) * 2^-24 * (double)((float)to - (float)from) + (double)(float)from)
// (ATen uniform_real_distribution<float> with its double accumulate type).
//
// One workgroup per job: the 624-word state lives in LDS; each regeneration ("twist") runs in three
// barrier-separated phases (words [0, 227) read only old words; [227, 454) read words of the first phase;
// [454, 624) read words of the second, the last word also word 0), 256 lanes wide; skipped draws only twist,
// drawn ones are tempered and written by the lane that owns their position.
#include <hip/hip_runtime.h>

#include "kernels.h"

namespace pt {
namespace dev {

constexpr int kMtN = 624, kMtM = 397, kInitThreads = 256;

__device__ __forceinline__ uint32_t mt_mix(uint32_t a, uint32_t b, uint32_t far) {
    const uint32_t y = (a & 0x80000000u) | (b & 0x7fffffffu);
    return far ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
}
__device__ __forceinline__ uint32_t mt_temper(uint32_t y) {
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
}

// the whole state regenerated in place (the standard next_state order, three dependency phases)
__device__ __forceinline__ void mt_twist(uint32_t *s) {
    const int t = threadIdx.x;
    uint32_t v = 0;
    // phase 1: k in [0, 227): s[k + 397], s[k], s[k + 1] all old
    if (t < kMtN - kMtM) v = mt_mix(s[t], s[t + 1], s[t + kMtM]);
    __syncthreads();
    if (t < kMtN - kMtM) s[t] = v;
    __syncthreads();
    // phase 2: k in [227, 454): s[k - 227] new (phase 1), s[k], s[k + 1] old
    {
        const int k = t + (kMtN - kMtM);
        if (k < 2 * (kMtN - kMtM)) v = mt_mix(s[k], s[k + 1], s[k - (kMtN - kMtM)]);
        __syncthreads();
        if (k < 2 * (kMtN - kMtM)) s[k] = v;
        __syncthreads();
    }
    // phase 3: k in [454, 624): s[k - 227] new (phase 2); the last word wraps to the new s[0]
    {
        const int k = t + 2 * (kMtN - kMtM);
        if (k < kMtN) v = mt_mix(s[k], k + 1 < kMtN ? s[k + 1] : s[0], s[k - (kMtN - kMtM)]);
        __syncthreads();
        if (k < kMtN) s[k] = v;
        __syncthreads();
    }
}

__global__ __launch_bounds__(kInitThreads) void k_torch_init(const pt_torch_init_job *__restrict__ jobs, int64_t n) {
    __shared__ uint32_t s[kMtN];
    const int64_t j = blockIdx.x;
    if (j >= n) return;
    const pt_torch_init_job &J = jobs[j];
    const int t = threadIdx.x;
    if (t == 0) {   // init_genrand(seed mod 2^32): a serial recurrence, one lane
        uint32_t x = (uint32_t)J.seed;
        s[0] = x;
        for (int i = 1; i < kMtN; ++i) {
            x = 1812433253u * (x ^ (x >> 30)) + (uint32_t)i;
            s[i] = x;
        }
    }
    __syncthreads();
    // the first output comes from the first twist (the generator starts with its state exhausted)
    int64_t skip = J.skip;
    mt_twist(s);
    while (skip >= kMtN) {   // whole skipped blocks: twist only
        mt_twist(s);
        skip -= kMtN;
    }
    int pos = (int)skip;   // next output index in the current block
    int tab = 0;
    int64_t done = 0;      // elements of table `tab` written
    while (tab < J.ntab) {
        const int64_t numel = J.numel[tab];
        if (done >= numel) {
            ++tab;
            done = 0;
            continue;
        }
        // outputs [pos, 624) of this block go to elements [done, done + 624 - pos) of the table
        const int64_t take = numel - done < (int64_t)(kMtN - pos) ? numel - done : (int64_t)(kMtN - pos);
        const float from = (float)J.lo[tab], to = (float)J.hi[tab];
        const double span = (double)(to - from), base = (double)from;
        float *out = J.out[tab] + done;
        for (int i = t; i < take; i += kInitThreads) {
            const uint32_t x = mt_temper(s[pos + i]) & 0xffffffu;
            out[i] = (float)((double)x * 0x1p-24 * span + base);
        }
        done += take;
        pos += (int)take;
        if (pos == kMtN) {
            __syncthreads();   // every lane has read the block
            mt_twist(s);
            pos = 0;
        }
    }
}

}  // namespace dev

hipError_t launch_torch_init(const pt_torch_init_job *d_jobs, int64_t n, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(dev::k_torch_init, dim3((unsigned)n), dim3(dev::kInitThreads), 0, st, d_jobs, n);
    return hipGetLastError();
}

}  // namespace pt
