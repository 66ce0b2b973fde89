// Measurement tool (not product code): the cost of splitting one universe's training over a TEAM of workgroups.
// A team is a leader and W-1 helpers on one XCD (workgroups b, b + 8, b + 16, ... of one launch: the dispatcher
// places workgroup i on XCD i % 8). Every "step" does what a split universe step would have to add to today's
// one-workgroup step:
//   helpers -> leader : each helper stores its step's payload (row ids / gradient words, `words` dwords, sc1
//                       write-through stores), waits for them (vmcnt(0)), then one lane adds to the leader's
//                       agent-scope arrival counter;
//   leader            : polls the counter (sc1 loads) until every helper of the step has arrived, reads all
//                       payloads (sc1 loads), stores its own `words` dwords (the updated rows the helpers read next)
//                       and publishes the next step number (sc1 store after vmcnt(0));
//   helpers           : poll that number, read the leader's words (sc1), start the next step.
// The guide's hand-off protocol (MI355X_MICROARCH.md, "Hand-offs measured with sc1 loads": sc1 stores, vmcnt(0),
// agent atomic / sc1 flag, sc1 polls, a workgroup barrier between the poll and the loads). No work between the
// exchanges: the result is the pure per-step exchange latency in shader-clock cycles (leader's clock64).
//
//   hipcc -O3 --offload-arch=gfx950 -o handoff_bench tools_gpu/handoff_bench.hip && ./handoff_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

struct Team {
    unsigned *arrive;     // [teams] helper arrivals (monotonic)
    unsigned *go;         // [teams] step number published by the leader
    unsigned *payload;    // [teams][W][words]
    unsigned long long *cycles;   // [teams] leader cycles over the timed steps
    unsigned *sink;       // [teams * 1024] keeps the loads live
};

__device__ __forceinline__ unsigned ld_sc1(const unsigned *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(unsigned *p, unsigned v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(1024, 1) void k_team(Team T, int W, int words, int steps, int warm) {
    const int team = blockIdx.x % 8, member = blockIdx.x / 8;   // one team per XCD, members on the same XCD
    const int tid = threadIdx.x;
    __shared__ unsigned s_flag;
    unsigned acc = 0;
    unsigned long long t0 = 0;
    unsigned *mine = T.payload + ((size_t)team * W + member) * words;
    for (int s = 1; s <= steps + warm; ++s) {
        if (s == warm + 1) t0 = clock64();
        if (member > 0) {
            // helper: payload, drain, arrive
            for (int i = tid; i < words; i += blockDim.x) st_sc1(mine + i, (unsigned)(s * 131 + i));
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (tid == 0) __hip_atomic_fetch_add(T.arrive + team, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            // wait for the leader's next step
            if (tid == 0) {
                while (ld_sc1(T.go + team) < (unsigned)s) __builtin_amdgcn_s_sleep(1);
            }
            __syncthreads();
            const unsigned *lead = T.payload + (size_t)team * W * words;
            for (int i = tid; i < words; i += blockDim.x) acc += ld_sc1(lead + i);
        } else {
            // leader: wait for every helper of step s, read their payloads, publish its own words and step s
            if (tid == 0) {
                const unsigned want = (unsigned)(s * (W - 1));
                while (ld_sc1(T.arrive + team) < want) __builtin_amdgcn_s_sleep(1);
            }
            __syncthreads();
            for (int m = 1; m < W; ++m)
                for (int i = tid; i < words; i += blockDim.x) acc += ld_sc1(T.payload + ((size_t)team * W + m) * words + i);
            for (int i = tid; i < words; i += blockDim.x) st_sc1(mine + i, acc + i);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (tid == 0) st_sc1(T.go + team, (unsigned)s);
        }
    }
    if (member == 0 && tid == 0) T.cycles[team] = clock64() - t0;
    T.sink[blockIdx.x * 1024 + tid] = acc;
    (void)s_flag;
}

int main(int argc, char **argv) {
    const int steps = argc > 1 ? atoi(argv[1]) : 3500, warm = 50;
    printf("{\"steps\": %d, \"results\": [", steps);
    bool first = true;
    for (int W : {2, 4}) {
        for (int words : {64, 1024, 4096}) {
            Team T;
            CK(hipMalloc(&T.arrive, 8 * sizeof(unsigned)));
            CK(hipMalloc(&T.go, 8 * sizeof(unsigned)));
            CK(hipMalloc(&T.payload, (size_t)8 * W * words * sizeof(unsigned)));
            CK(hipMalloc(&T.cycles, 8 * sizeof(unsigned long long)));
            CK(hipMalloc(&T.sink, (size_t)8 * W * 1024 * sizeof(unsigned)));
            CK(hipMemset(T.arrive, 0, 8 * sizeof(unsigned)));
            CK(hipMemset(T.go, 0, 8 * sizeof(unsigned)));
            hipEvent_t a, b;
            CK(hipEventCreate(&a));
            CK(hipEventCreate(&b));
            CK(hipEventRecord(a, 0));
            // 8 teams x W members = 8W workgroups, one per CU: all resident at once
            hipLaunchKernelGGL(k_team, dim3(8 * W), dim3(1024), 0, 0, T, W, words, steps, warm);
            CK(hipGetLastError());
            CK(hipEventRecord(b, 0));
            CK(hipDeviceSynchronize());
            float ms = 0;
            CK(hipEventElapsedTime(&ms, a, b));
            std::vector<unsigned long long> cyc(8);
            CK(hipMemcpy(cyc.data(), T.cycles, 8 * sizeof(unsigned long long), hipMemcpyDeviceToHost));
            double mean = 0;
            for (auto c : cyc) mean += (double)c / 8;
            printf("%s{\"W\": %d, \"words\": %d, \"cycles_per_step\": %.0f, \"us_per_step_wall\": %.3f}", first ? "" : ", ",
                   W, words, mean / steps, 1e3 * ms / (steps + warm));
            first = false;
            CK(hipFree(T.arrive)); CK(hipFree(T.go)); CK(hipFree(T.payload)); CK(hipFree(T.cycles)); CK(hipFree(T.sink));
        }
    }
    printf("]}\n");
    return 0;
}
