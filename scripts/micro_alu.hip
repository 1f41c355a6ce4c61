// micro_alu.hip -- gfx950 issue-rate probe for the integer ops the WAF prefilter hash can use,
// and for random-address LDS reads.  Standalone: hipcc --offload-arch=gfx950 -O3 micro_alu.hip.
// Prints lane-ops/s per instruction; full rate on MI355X ~= 256 CU * 64 lanes * clock.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define CHAINS 8
#define ITERS 2048

#define DEF_KERNEL(NAME, ASM)                                                                        \
    __global__ void NAME(uint32_t *out, uint32_t seed) {                                            \
        uint32_t x[CHAINS];                                                                          \
        for (int c = 0; c < CHAINS; c++) x[c] = threadIdx.x * 7919u + c * 104729u + seed;           \
        const uint32_t k = seed | 0x9E3779B1u;                                                       \
        for (int i = 0; i < ITERS; i++) {                                                            \
            _Pragma("unroll") for (int c = 0; c < CHAINS; c++) asm volatile(ASM : "+v"(x[c]) : "v"(k)); \
        }                                                                                            \
        uint32_t s = 0;                                                                              \
        for (int c = 0; c < CHAINS; c++) s ^= x[c];                                                  \
        if (s == 0x12345678u) out[0] = s;                                                            \
    }

DEF_KERNEL(k_mul_lo, "v_mul_lo_u32 %0, %0, %1")
DEF_KERNEL(k_mul_hi, "v_mul_hi_u32 %0, %0, %1")
DEF_KERNEL(k_mul_u24, "v_mul_u32_u24 %0, %0, %1")
DEF_KERNEL(k_mul_hi_u24, "v_mul_hi_u32_u24 %0, %0, %1")
DEF_KERNEL(k_xor, "v_xor_b32 %0, %0, %1")
DEF_KERNEL(k_lshl_or, "v_lshl_or_b32 %0, %1, %0, %0")
DEF_KERNEL(k_bfe, "v_bfe_u32 %0, %0, %1, 5")
DEF_KERNEL(k_bitop3, "v_bitop3_b32 %0, %0, %1, %0 bitop3:0x6c")
DEF_KERNEL(k_alignbyte, "v_alignbyte_b32 %0, %0, %1, 1")
DEF_KERNEL(k_perm, "v_perm_b32 %0, %0, %1, %1")
DEF_KERNEL(k_pk_mul16, "v_pk_mul_lo_u16 %0, %0, %1")
DEF_KERNEL(k_pk_lshl16, "v_pk_lshlrev_b16 %0, %0, %1")
DEF_KERNEL(k_min3, "v_min3_u32 %0, %0, %1, %0")
DEF_KERNEL(k_dot4, "v_dot4_u32_u8 %0, %0, %1, %0")
DEF_KERNEL(k_lshl_add, "v_lshl_add_u32 %0, %0, 3, %1")
DEF_KERNEL(k_and_or, "v_and_or_b32 %0, %0, %1, %0")
DEF_KERNEL(k_bfi, "v_bfi_b32 %0, %1, %0, %1")
DEF_KERNEL(k_lshr, "v_lshrrev_b32 %0, 7, %0")
DEF_KERNEL(k_mad_u24, "v_mad_u32_u24 %0, %0, %1, %1")
DEF_KERNEL(k_pk_mad16, "v_pk_mad_u16 %0, %0, %1, %1")

__global__ void k_mad64(uint32_t *out, uint32_t seed) {
    uint64_t x[CHAINS];
    for (int c = 0; c < CHAINS; c++) x[c] = threadIdx.x * 7919u + c * 104729u + seed;
    const uint32_t k = seed | 0x9E3779B1u;
    for (int i = 0; i < ITERS; i++) {
#pragma unroll
        for (int c = 0; c < CHAINS; c++) {
            uint32_t lo = (uint32_t)x[c];
            asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, 0" : "=v"(x[c]) : "v"(lo), "v"(k) : "vcc");
        }
    }
    uint32_t s = 0;
    for (int c = 0; c < CHAINS; c++) s ^= (uint32_t)x[c];
    if (s == 0x12345678u) out[0] = s;
}

// random LDS reads: each lane walks its own hash chain through a 128 KiB table
template <int B64>
__global__ __launch_bounds__(1024) void k_lds(uint32_t *out, uint32_t seed) {
    extern __shared__ uint32_t lds[];
    for (uint32_t i = threadIdx.x; i < 32768; i += 1024) lds[i] = i * 2654435761u;
    __syncthreads();
    uint32_t x[CHAINS];
    for (int c = 0; c < CHAINS; c++) x[c] = (threadIdx.x * 7919u + c * 104729u + seed);
    for (int i = 0; i < ITERS / 4; i++) {
#pragma unroll
        for (int c = 0; c < CHAINS; c++) {
            if (B64) {
                const uint2 v = reinterpret_cast<const uint2 *>(lds)[(x[c] >> 3) & 16383];
                x[c] += v.x ^ v.y;
            } else {
                x[c] += lds[(x[c] >> 3) & 32767];
            }
        }
    }
    uint32_t s = 0;
    for (int c = 0; c < CHAINS; c++) s ^= x[c];
    if (s == 0x12345678u) out[0] = s;
}

int main() {
    uint32_t *d;
    (void)hipMalloc(&d, 64);
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    hipEvent_t a, b;
    (void)hipEventCreate(&a); (void)hipEventCreate(&b);
    const int blocks = cus * 8, threads = 256;
    struct K { const char *name; void (*f)(uint32_t *, uint32_t); } ks[] = {
        {"v_mul_lo_u32", k_mul_lo}, {"v_mul_hi_u32", k_mul_hi}, {"v_mul_u32_u24", k_mul_u24},
        {"v_mul_hi_u32_u24", k_mul_hi_u24}, {"v_xor_b32", k_xor}, {"v_lshl_or_b32", k_lshl_or},
        {"v_bfe_u32", k_bfe}, {"v_bitop3_b32", k_bitop3}, {"v_alignbyte_b32", k_alignbyte},
        {"v_perm_b32", k_perm}, {"v_mad_u64_u32", k_mad64},
        {"v_pk_mul_lo_u16", k_pk_mul16}, {"v_pk_lshlrev_b16", k_pk_lshl16}, {"v_min3_u32", k_min3},
        {"v_dot4_u32_u8", k_dot4}, {"v_lshl_add_u32", k_lshl_add}, {"v_and_or_b32", k_and_or},
        {"v_bfi_b32", k_bfi}, {"v_lshrrev_b32", k_lshr}, {"v_mad_u32_u24", k_mad_u24}, {"v_pk_mad_u16", k_pk_mad16}};
    for (auto &k : ks) {
        hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, d, 1u);
        (void)hipEventRecord(a);
        for (int r = 0; r < 5; r++) hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, d, (uint32_t)r);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        const double ops = 5.0 * blocks * threads * (double)CHAINS * ITERS;
        printf("%-18s %8.2f T lane-ops/s\n", k.name, ops / (ms * 1e-3) / 1e12);
    }
    (void)hipFuncSetAttribute((const void *)k_lds<0>, hipFuncAttributeMaxDynamicSharedMemorySize, 131072);
    (void)hipFuncSetAttribute((const void *)k_lds<1>, hipFuncAttributeMaxDynamicSharedMemorySize, 131072);
    for (int b64 = 0; b64 < 2; b64++) {
        auto f = b64 ? k_lds<1> : k_lds<0>;
        hipLaunchKernelGGL(f, dim3(cus), dim3(1024), 131072, 0, d, 1u);
        (void)hipEventRecord(a);
        for (int r = 0; r < 5; r++) hipLaunchKernelGGL(f, dim3(cus), dim3(1024), 131072, 0, d, (uint32_t)r);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        const double reads = 5.0 * cus * 1024 * (double)CHAINS * (ITERS / 4);
        printf("ds_read_b%d random  %8.2f T lane-reads/s  (%.2f per CU per clock @2.4GHz)\n", b64 ? 64 : 32,
               reads / (ms * 1e-3) / 1e12, reads / (ms * 1e-3) / cus / 2.4e9);
    }
    return 0;
}
