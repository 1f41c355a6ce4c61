// micro_lds.hip -- gfx950 random-address LDS read rates for the WAF Bloom probe shapes, and what
// an unaligned ds_read_b32 returns.  Standalone: hipcc --offload-arch=gfx950 -O3 micro_lds.hip.
// Each lane issues 8 independent reads per iteration at hashed addresses inside 128 KiB (the
// scan's shape: 8 probes in flight per lane, 16 waves per CU).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define ITERS 4096

template <int KIND>   // 0: b32 aligned, 1: b64 aligned, 2: b32 at any byte address, 3: b128 aligned, 4: u16
__global__ __launch_bounds__(1024) void k_lds(uint32_t *out, uint32_t seed) {
    extern __shared__ uint32_t lds[];
    for (uint32_t i = threadIdx.x; i < 32768 + 64; i += 1024) lds[i] = i * 2654435761u;
    __syncthreads();
    uint32_t x = threadIdx.x * 0x9E3779B1u + seed, acc = 0;
    const uint8_t *lb = reinterpret_cast<const uint8_t *>(lds);
    for (int i = 0; i < ITERS; i++) {
        uint32_t v[8];
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const uint32_t h = (x + j * 0x7F4A7C15u) * 0x85EBCA77u;
            if (KIND == 0) v[j] = lds[h >> 17];
            else if (KIND == 1) { const uint2 q = reinterpret_cast<const uint2 *>(lds)[h >> 18]; v[j] = q.x ^ q.y; }
            else if (KIND == 2) { uint32_t t; __builtin_memcpy(&t, lb + (h >> 15), 4); v[j] = t; }
            else if (KIND == 3) { const uint4 q = reinterpret_cast<const uint4 *>(lds)[h >> 19]; v[j] = q.x ^ q.y ^ q.z ^ q.w; }
            else v[j] = reinterpret_cast<const uint16_t *>(lds)[h >> 16];
        }
#pragma unroll
        for (int j = 0; j < 8; j++) acc ^= v[j];
        x += acc | 1u;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

__global__ void k_unaligned(uint32_t *out) {
    __shared__ uint32_t lds[16];
    if (threadIdx.x < 16) lds[threadIdx.x] = 0x03020100u + threadIdx.x * 0x04040404u;
    __syncthreads();
    if (threadIdx.x < 4) {
        const uint8_t *lb = reinterpret_cast<const uint8_t *>(lds);
        uint32_t t;
        __builtin_memcpy(&t, lb + 4 + threadIdx.x, 4);
        out[threadIdx.x] = t;
        // an explicitly dword-typed access at a misaligned address
        out[4 + threadIdx.x] = *reinterpret_cast<const uint32_t *>(lb + 4 + threadIdx.x);
    }
}

int main() {
    uint32_t *d;
    (void)hipMalloc(&d, 64);
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    hipEvent_t a, b;
    (void)hipEventCreate(&a); (void)hipEventCreate(&b);
    const char *names[] = {"ds_read_b32 random", "ds_read_b64 random", "b32 any byte addr", "ds_read_b128 random", "ds_read_u16 random"};
    void (*fs[])(uint32_t *, uint32_t) = {k_lds<0>, k_lds<1>, k_lds<2>, k_lds<3>, k_lds<4>};
    for (int k = 0; k < 5; k++) {
        (void)hipFuncSetAttribute((const void *)fs[k], hipFuncAttributeMaxDynamicSharedMemorySize, 131072 + 256);
        hipLaunchKernelGGL(fs[k], dim3(cus), dim3(1024), 131072 + 256, 0, d, 1u);
        (void)hipEventRecord(a);
        for (int r = 0; r < 5; r++) hipLaunchKernelGGL(fs[k], dim3(cus), dim3(1024), 131072 + 256, 0, d, (uint32_t)r);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        const double instr = 5.0 * cus * 16 * (double)ITERS * 8;   // wave-instructions
        printf("%-22s %7.3f ms  %6.2f CU-cycles per wave-instruction @2.4GHz\n", names[k], ms,
               ms * 1e-3 * 2.4e9 * cus / instr);
    }
    hipLaunchKernelGGL(k_unaligned, dim3(1), dim3(64), 0, 0, d);
    uint32_t h[8];
    (void)hipMemcpy(h, d, 32, hipMemcpyDeviceToHost);
    printf("unaligned b32 reads at byte 4..7 (memcpy): %08x %08x %08x %08x\n", h[0], h[1], h[2], h[3]);
    printf("unaligned b32 reads at byte 4..7 (typed):  %08x %08x %08x %08x\n", h[4], h[5], h[6], h[7]);
    return 0;
}
