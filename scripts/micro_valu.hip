// VALU issue cost per wave-instruction on gfx950 for the ops of the scan's probe (k_waf_scan):
// each lane runs 16 independent chains of one op, 8 waves per SIMD; the time per op is reported
// relative to v_and_b32.  Timing only (no result is checked beyond keeping it live).
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/micro_valu scripts/micro_valu.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int ITERS = 4096;

#define CHAINS(OP)                                                                                     \
    _Pragma("unroll") for (int k = 0; k < 16; k++) { OP; }

template <int KIND>
__global__ __launch_bounds__(1024) void k_micro(uint32_t *out, uint32_t c) {
    uint32_t x[16];
    uint64_t y[16];
#pragma unroll
    for (int k = 0; k < 16; k++) { x[k] = threadIdx.x * 977u + k; y[k] = x[k]; }
    for (int it = 0; it < ITERS; it++) {
        if constexpr (KIND == 0) CHAINS(asm volatile("v_and_b32 %0, %1, %0" : "+v"(x[k]) : "s"(c)))
        if constexpr (KIND == 1) CHAINS(asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %2, 0" : "=v"(y[k]) : "v"((uint32_t)y[k]), "s"(c) : "s0", "s1"))
        if constexpr (KIND == 2) CHAINS(asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x[k]) : "s"(c)))
        if constexpr (KIND == 3) CHAINS(asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(x[k]) : "s"(c)))
        if constexpr (KIND == 4) CHAINS(asm volatile("v_mul_u32_u24 %0, %1, %0" : "+v"(x[k]) : "s"(c)))
        if constexpr (KIND == 5) CHAINS(asm volatile("v_mul_hi_u32_u24 %0, %1, %0" : "+v"(x[k]) : "s"(c)))
        if constexpr (KIND == 6) CHAINS(asm volatile("v_perm_b32 %0, %1, %0, %0" : "+v"(x[k]) : "s"(c)))
        if constexpr (KIND == 7) CHAINS(asm volatile("v_bitop3_b32 %0, %0, %1, %0 bitop3:0x30" : "+v"(x[k]) : "s"(c)))
        if constexpr (KIND == 8) CHAINS(asm volatile("v_alignbyte_b32 %0, %0, %1, 2" : "+v"(x[k]) : "s"(c)))
        if constexpr (KIND == 9) CHAINS(asm volatile("v_cmp_eq_u32_e64 s[2:3], %0, %1\n\tv_cndmask_b32_e64 %0, %0, %1, s[2:3]" : "+v"(x[k]) : "v"(c) : "s2", "s3"))
        if constexpr (KIND == 10) CHAINS(asm volatile("v_cndmask_b32_e64 %0, %0, %1, s[2:3]" : "+v"(x[k]) : "v"(c) : "s2", "s3"))
        if constexpr (KIND == 11) CHAINS(asm volatile("v_mul_lo_u16 %0, %0, %1" : "+v"(x[k]) : "s"(c)))
        if constexpr (KIND == 12) CHAINS(asm volatile("v_xad_u32 %0, %0, %1, %0" : "+v"(x[k]) : "s"(c)))
        if constexpr (KIND == 13) CHAINS(asm volatile("v_mad_u32_u24 %0, %0, %1, %0" : "+v"(x[k]) : "s"(c)))
        if constexpr (KIND == 14) CHAINS(asm volatile("v_pk_mul_lo_u16 %0, %0, %1" : "+v"(x[k]) : "s"(c)))
        if constexpr (KIND == 15) CHAINS(asm volatile("v_lshl_add_u32 %0, %0, 5, %1" : "+v"(x[k]) : "s"(c)))
    }
    uint32_t s = 0;
#pragma unroll
    for (int k = 0; k < 16; k++) s ^= x[k] ^ (uint32_t)y[k] ^ (uint32_t)(y[k] >> 32);
    if (s == 0x12345678u) out[0] = s;
}

static const char *NAMES[] = {"v_and_b32", "v_mad_u64_u32", "v_mul_lo_u32", "v_mul_hi_u32", "v_mul_u32_u24",
                              "v_mul_hi_u32_u24", "v_perm_b32", "v_bitop3_b32", "v_alignbyte_b32",
                              "v_cmp_e64+v_cndmask (2 ops)", "v_cndmask_b32_e64", "v_mul_lo_u16", "v_xad_u32",
                              "v_mad_u32_u24", "v_pk_mul_lo_u16", "v_lshl_add_u32"};

template <int K>
float run(uint32_t *d, int blocks) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a); (void)hipEventCreate(&b);
    k_micro<K><<<blocks, 1024>>>(d, 3u);
    (void)hipEventRecord(a);
    k_micro<K><<<blocks, 1024>>>(d, 3u);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms;
}

int main() {
    uint32_t *d;
    if (hipMalloc(&d, 64) != hipSuccess) return 1;
    hipDeviceProp_t p;
    (void)hipGetDeviceProperties(&p, 0);
    const int blocks = p.multiProcessorCount * 2;   // 8 waves per SIMD
    float t[16];
    t[0] = run<0>(d, blocks); t[1] = run<1>(d, blocks); t[2] = run<2>(d, blocks); t[3] = run<3>(d, blocks);
    t[4] = run<4>(d, blocks); t[5] = run<5>(d, blocks); t[6] = run<6>(d, blocks); t[7] = run<7>(d, blocks);
    t[8] = run<8>(d, blocks); t[9] = run<9>(d, blocks); t[10] = run<10>(d, blocks); t[11] = run<11>(d, blocks);
    t[12] = run<12>(d, blocks); t[13] = run<13>(d, blocks); t[14] = run<14>(d, blocks); t[15] = run<15>(d, blocks);
    // wave-instructions per SIMD: blocks * 16 waves / (4 SIMDs * CUs) * ITERS * 16
    const double wi = (double)blocks * 16 / (4.0 * p.multiProcessorCount) * ITERS * 16;
    const double clk = p.clockRate * 1e3;   // Hz
    printf("CUs %d clock %.0f MHz\n", p.multiProcessorCount, clk / 1e6);
    for (int k = 0; k < 16; k++)
        printf("%-30s %8.3f ms  %6.2f cycles/wave-instr  x%.2f of v_and\n", NAMES[k], t[k], t[k] * 1e-3 * clk / wi,
               t[k] / t[0]);
    (void)hipFree(d);
    return 0;
}
