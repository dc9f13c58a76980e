// Cross-attention streaming lab: how fast can one wave per (row, head) stream its clip's K/V
// (T keys x 128 B each for K and for V, head-major) with no math, by staging route and depth?
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/lab_attn.hip -o /tmp/lab_attn && /tmp/lab_attn
// Variants (all consume every byte: an xor of the staged words is written out):
//   lds<D>: global_load_lds 16 B per lane into a D-deep LDS ring of 64-key chunks (the product's route)
//   reg<D>: global_load_dwordx4 into registers, D chunks in flight (no LDS)
// Not part of the product: a measurement tool for k_attn_step's design.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            fprintf(stderr, "HIP %s at %d: %s\n", hipGetErrorString(e_), __LINE__, #x);     \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

typedef __attribute__((address_space(3))) void * lds_ptr_t;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// lds<D>: per chunk 8 + 8 global_load_lds of 1 KB; wait for chunk c, read it (one 16 B word per lane
// per KB), refill
template <int D, int AUX>
__global__ __launch_bounds__(64) void k_lds(const char * __restrict__ kv, int T, uint32_t * out) {
    __shared__ __attribute__((aligned(1024))) char smem[D * 16384];
    const int lane = threadIdx.x;
    const size_t item = blockIdx.y * gridDim.x + blockIdx.x;
    const char * kh = kv + item * (size_t) T * 128;
    const char * vh = kv + ((size_t) gridDim.x * gridDim.y + item) * (size_t) T * 128;
    const int nch = T / 64;
    auto stage = [&](int b, int c) {
        char * s = smem + b * 16384;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const size_t off = (size_t) c * 8192 + i * 1024 + lane * 16;
            __builtin_amdgcn_global_load_lds((const void *) (kh + off), (lds_ptr_t) (s + i * 1024), 16, 0, AUX);
            __builtin_amdgcn_global_load_lds((const void *) (vh + off), (lds_ptr_t) (s + 8192 + i * 1024), 16, 0, AUX);
        }
    };
    uint32_t x = 0;
#pragma unroll
    for (int c = 0; c < D; ++c)
        if (c < nch) stage(c, c);
    for (int c = 0; c < nch; ++c) {
        const int ahead = min(D - 1, nch - 1 - c);
        // chunk c landed once at most `ahead` chunks (16 loads each) are outstanding
        static_assert(D <= 4, "vmcnt holds at most 63 outstanding loads");
        if (ahead == 3) wait_vmcnt<16 * 3>();
        else if (ahead == 2) wait_vmcnt<16 * 2>();
        else if (ahead == 1) wait_vmcnt<16>();
        else wait_vmcnt<0>();
        const char * s = smem + (c % D) * 16384;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const u32x4 w = *(const u32x4 *) (s + i * 1024 + lane * 16);
            x ^= w.x ^ w.y ^ w.z ^ w.w;
        }
        if (c + D < nch) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            stage(c % D, c + D);
        }
    }
    out[item * 64 + lane] = x;
}

// reg<D>: D chunks of 16 KB in flight in registers (16 dwordx4 per lane per chunk)
template <int D, bool NT>
__global__ __launch_bounds__(64) void k_reg(const char * __restrict__ kv, int T, uint32_t * out) {
    const int lane = threadIdx.x;
    const size_t item = blockIdx.y * gridDim.x + blockIdx.x;
    const u32x4 * kh = (const u32x4 *) (kv + item * (size_t) T * 128);
    const u32x4 * vh = (const u32x4 *) (kv + ((size_t) gridDim.x * gridDim.y + item) * (size_t) T * 128);
    const int nch = T / 64;
    u32x4 buf[D][16];
    auto ld = [&](const u32x4 * p) { return NT ? __builtin_nontemporal_load(p) : *p; };
    auto stage = [&](u32x4 (&b)[16], int c) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            b[i] = ld(kh + (size_t) c * 512 + i * 64 + lane);
            b[8 + i] = ld(vh + (size_t) c * 512 + i * 64 + lane);
        }
    };
    uint32_t x = 0;
#pragma unroll
    for (int c = 0; c < D; ++c) stage(buf[c], c);
    for (int c0 = 0; c0 < nch; c0 += D) {
#pragma unroll
        for (int j = 0; j < D; ++j) {
            const int c = c0 + j;
            if (c < nch) {
#pragma unroll
                for (int i = 0; i < 16; ++i) x ^= buf[j][i].x ^ buf[j][i].y ^ buf[j][i].z ^ buf[j][i].w;
                if (c + D < nch) stage(buf[j], c + D);
            }
        }
    }
    out[item * 64 + lane] = x;
}

template <typename K>
float time_it(K launch, int iters) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int i = 0; i < iters; ++i) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return 1e3f * ms / iters;
}

int main() {
    const int H = 20, T = 1536;  // 1500 keys rounded to whole chunks
    const int NB = 8;            // rotate over NB copies so nothing stays in the MALL between launches
    const size_t per = (size_t) 2 * 32 * H * T * 128;
    char * buf;
    CK(hipMalloc(&buf, per * NB));
    CK(hipMemset(buf, 1, per * NB));
    uint32_t * out;
    CK(hipMalloc(&out, 32 * H * 64 * 4));
    for (int R : {1, 32}) {
        const double bytes = 2.0 * R * H * T * 128;
        auto run = [&](const char * name, auto kern) {
            int it = 0;
            const float us = time_it([&] {
                hipLaunchKernelGGL(kern, dim3(H, R), dim3(64), 0, 0, buf + per * (it++ % NB), T, out);
            }, 40);
            printf("{\"rows\": %d, \"variant\": \"%s\", \"us\": %.2f, \"GBps\": %.0f}\n", R, name, us, bytes / us / 1e3);
        };
        run("lds2", k_lds<2, 2>);
        run("lds3", k_lds<3, 2>);
        run("lds3_temporal", k_lds<3, 0>);
        run("lds4", k_lds<4, 2>);
        run("reg2", k_reg<2, true>);
        run("reg3", k_reg<3, true>);
        run("reg3_temporal", k_reg<3, false>);
        run("reg4", k_reg<4, true>);
    }
    return 0;
}
