// Stream-overlap lab: can a bandwidth-bound launch (the decode pass's cross attention: 320 blocks of 128
// threads streaming 384 KB each) run beside a chain of latency-bound launches (decode-row GEMMs: 80 blocks
// of 512 threads, ~40 KB each, 10 dependent launches) on another stream? Times, per repetition:
//   X alone, the chain alone, both issued on two streams (eager), both as two graphs on two streams, and
//   one graph with the two as parallel branches (fork/join by events during capture).
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/lab_overlap.hip -o /tmp/lab_overlap && /tmp/lab_overlap
// Not part of the product: a measurement tool for the decode-pass design.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            fprintf(stderr, "HIP %s at %d: %s\n", hipGetErrorString(e_), __LINE__, #x);     \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

typedef float float4v __attribute__((ext_vector_type(4)));

// each block streams `per` bytes (non-temporal 16-B loads), LDS-free like the DMA ring's consumer
__global__ __launch_bounds__(128) void k_stream(const float4v * __restrict__ src, size_t per16, float * out) {
    const float4v * p = src + (size_t) blockIdx.x * per16;
    float4v acc = {0, 0, 0, 0};
    for (size_t i = threadIdx.x; i < per16; i += 4 * 128) {
        float4v a = __builtin_nontemporal_load(p + i);
        float4v b = i + 128 < per16 ? __builtin_nontemporal_load(p + i + 128) : float4v{0, 0, 0, 0};
        float4v c = i + 256 < per16 ? __builtin_nontemporal_load(p + i + 256) : float4v{0, 0, 0, 0};
        float4v d = i + 384 < per16 ? __builtin_nontemporal_load(p + i + 384) : float4v{0, 0, 0, 0};
        acc += a + b + c + d;
    }
    const float s = acc.x + acc.y + acc.z + acc.w;
    if (s == 12345.678f) out[blockIdx.x] = s;  // keeps the loads
}

// compute only: the same grid spinning on VALU for about as long as k_stream takes (no memory traffic)
__global__ __launch_bounds__(128) void k_spin(int iters, float * out) {
    float a = threadIdx.x, b = 1.0001f;
    for (int i = 0; i < iters; ++i) a = a * b + 0.5f;
    if (a == 12345.678f) out[blockIdx.x] = a;
}

// a latency-bound stage: each block reads its slice, reduces across 8 waves through LDS, writes a row
__global__ __launch_bounds__(512) void k_small(const float4v * __restrict__ w, size_t per16, const float * in, float * out) {
    __shared__ float red[8];
    const float4v * p = w + (size_t) blockIdx.x * per16;
    float4v acc = {0, 0, 0, 0};
    for (size_t i = threadIdx.x; i < per16; i += 512) acc += __builtin_nontemporal_load(p + i);
    float s = acc.x + acc.y + acc.z + acc.w + in[blockIdx.x & 63];
    for (int o = 32; o; o >>= 1) s += __shfl_xor(s, o);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        float t = 0;
        for (int i = 0; i < 8; ++i) t += red[i];
        out[blockIdx.x & 63] = t * 1e-9f;
    }
}

int main() {
    const int NX = 320, NG = 80, CH = 10;
    const size_t xper = 384 * 1024 / 16, gper = 40 * 1024 / 16;
    float4v *xs, *ws;
    float *xo, *ga, *gb;
    CK(hipMalloc(&xs, NX * xper * 16 * 2));  // two buffers: consecutive X launches miss the MALL
    CK(hipMalloc(&ws, (size_t) CH * NG * gper * 16 * 2));
    CK(hipMalloc(&xo, 4096));
    CK(hipMalloc(&ga, 4096));
    CK(hipMalloc(&gb, 4096));
    CK(hipMemset(xs, 0, NX * xper * 16 * 2));
    CK(hipMemset(ws, 0, (size_t) CH * NG * gper * 16 * 2));
    CK(hipMemset(ga, 0, 4096));
    hipStream_t s1, s2;
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    hipEvent_t e0, e1, fork, join;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&join, hipEventDisableTiming));
    int it = 0;
    auto X = [&](hipStream_t s) {
        k_stream<<<NX, 128, 0, s>>>(xs + (size_t) (it & 1) * NX * xper, xper, xo);
    };
    auto G = [&](hipStream_t s) {
        for (int c = 0; c < CH; ++c)
            k_small<<<NG, 512, 0, s>>>(ws + ((size_t) (it & 1) * CH + c) * NG * gper, gper, c & 1 ? gb : ga, c & 1 ? ga : gb);
    };
    auto timeit = [&](const char * name, auto && body) {
        for (int w = 0; w < 5; ++w, ++it) body();
        CK(hipDeviceSynchronize());
        const int R = 50;
        CK(hipEventRecord(e0, s1));
        for (int r = 0; r < R; ++r, ++it) body();
        CK(hipEventRecord(fork, s2));
        CK(hipStreamWaitEvent(s1, fork, 0));
        CK(hipEventRecord(e1, s1));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("%-44s %8.2f us per repetition\n", name, 1000.0f * ms / R);
    };
    // everything below starts after e0 on s1; s2 joins s1 at each repetition start so the pair is aligned
    auto pair_eager = [&]() {
        CK(hipEventRecord(fork, s1));
        CK(hipStreamWaitEvent(s2, fork, 0));
        X(s1);
        G(s2);
        CK(hipEventRecord(join, s2));
        CK(hipStreamWaitEvent(s1, join, 0));
    };
    timeit("X alone (320 x 384 KB)", [&]() { X(s1); });
    timeit("chain alone (10 x 80 blocks)", [&]() { G(s1); });
    timeit("X then chain, one stream", [&]() { X(s1); G(s1); });
    timeit("X || chain, two streams, eager", pair_eager);
    // graphs: X graph on s1, chain graph on s2
    hipGraph_t gx, gg, gp;
    hipGraphExec_t ex[2], eg[2], ep[2];
    for (int b = 0; b < 2; ++b) {
        it = b;
        CK(hipStreamBeginCapture(s1, hipStreamCaptureModeThreadLocal));
        X(s1);
        CK(hipStreamEndCapture(s1, &gx));
        CK(hipGraphInstantiate(&ex[b], gx, nullptr, nullptr, 0));
        CK(hipStreamBeginCapture(s2, hipStreamCaptureModeThreadLocal));
        G(s2);
        CK(hipStreamEndCapture(s2, &gg));
        CK(hipGraphInstantiate(&eg[b], gg, nullptr, nullptr, 0));
        CK(hipStreamBeginCapture(s1, hipStreamCaptureModeThreadLocal));
        CK(hipEventRecord(fork, s1));
        CK(hipStreamWaitEvent(s2, fork, 0));
        X(s1);
        G(s2);
        CK(hipEventRecord(join, s2));
        CK(hipStreamWaitEvent(s1, join, 0));
        CK(hipStreamEndCapture(s1, &gp));
        CK(hipGraphInstantiate(&ep[b], gp, nullptr, nullptr, 0));
    }
    it = 0;
    timeit("chain alone, graph", [&]() { CK(hipGraphLaunch(eg[it & 1], s1)); });
    timeit("X || chain, two graphs on two streams", [&]() {
        CK(hipEventRecord(fork, s1));
        CK(hipStreamWaitEvent(s2, fork, 0));
        CK(hipGraphLaunch(ex[it & 1], s1));
        CK(hipGraphLaunch(eg[it & 1], s2));
        CK(hipEventRecord(join, s2));
        CK(hipStreamWaitEvent(s1, join, 0));
    });
    timeit("X || chain, one graph with two branches", [&]() { CK(hipGraphLaunch(ep[it & 1], s1)); });
    // what slows the chain beside X: memory traffic (a spinning X) or the grid size (X on 64 blocks)
    const int spin = 20000;
    timeit("spin alone (320 blocks, VALU only)", [&]() { k_spin<<<NX, 128, 0, s1>>>(spin, xo); });
    timeit("spin || chain, two streams, eager", [&]() {
        CK(hipEventRecord(fork, s1));
        CK(hipStreamWaitEvent(s2, fork, 0));
        k_spin<<<NX, 128, 0, s1>>>(spin, xo);
        G(s2);
        CK(hipEventRecord(join, s2));
        CK(hipStreamWaitEvent(s1, join, 0));
    });
    timeit("X64 alone (64 x 384 KB)", [&]() { k_stream<<<64, 128, 0, s1>>>(xs + (size_t) (it & 1) * NX * xper, xper, xo); });
    timeit("X64 || chain, two streams, eager", [&]() {
        CK(hipEventRecord(fork, s1));
        CK(hipStreamWaitEvent(s2, fork, 0));
        k_stream<<<64, 128, 0, s1>>>(xs + (size_t) (it & 1) * NX * xper, xper, xo);
        G(s2);
        CK(hipEventRecord(join, s2));
        CK(hipStreamWaitEvent(s1, join, 0));
    });
    printf("done\n");
    return 0;
}
