#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define N_ITERS 4096

__global__ __launch_bounds__(1024) void k_v_lshl_or_b32(uint32_t* out, uint32_t seed) {
    uint32_t a0 = seed ^ threadIdx.x, a1 = a0 * 3u, a2 = a0 * 5u, a3 = a0 * 7u, a4 = a0 * 11u, a5 = a0 * 13u, a6 = a0 * 17u, a7 = a0 * 19u;
    for (int i = 0; i < N_ITERS; ++i) {
        asm volatile("v_lshl_or_b32 %0, %1, 3, %0\nv_lshl_or_b32 %1, %2, 3, %1\nv_lshl_or_b32 %2, %3, 3, %2\nv_lshl_or_b32 %3, %4, 3, %3\nv_lshl_or_b32 %4, %5, 3, %4\nv_lshl_or_b32 %5, %6, 3, %5\nv_lshl_or_b32 %6, %7, 3, %6\nv_lshl_or_b32 %7, %0, 3, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc", "s0");
    }
    uint64_t r = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
    if ((uint32_t)r == 0x12345678u) out[blockIdx.x] = (uint32_t)r;
}
__global__ __launch_bounds__(1024) void k_v_lshlrev_b32(uint32_t* out, uint32_t seed) {
    uint32_t a0 = seed ^ threadIdx.x, a1 = a0 * 3u, a2 = a0 * 5u, a3 = a0 * 7u, a4 = a0 * 11u, a5 = a0 * 13u, a6 = a0 * 17u, a7 = a0 * 19u;
    for (int i = 0; i < N_ITERS; ++i) {
        asm volatile("v_lshlrev_b32 %0, 3, %1\nv_lshlrev_b32 %1, 3, %2\nv_lshlrev_b32 %2, 3, %3\nv_lshlrev_b32 %3, 3, %4\nv_lshlrev_b32 %4, 3, %5\nv_lshlrev_b32 %5, 3, %6\nv_lshlrev_b32 %6, 3, %7\nv_lshlrev_b32 %7, 3, %0" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc", "s0");
    }
    uint64_t r = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
    if ((uint32_t)r == 0x12345678u) out[blockIdx.x] = (uint32_t)r;
}
__global__ __launch_bounds__(1024) void k_v_lshlrev_b32_s(uint32_t* out, uint32_t seed) {
    uint32_t a0 = seed ^ threadIdx.x, a1 = a0 * 3u, a2 = a0 * 5u, a3 = a0 * 7u, a4 = a0 * 11u, a5 = a0 * 13u, a6 = a0 * 17u, a7 = a0 * 19u;
    for (int i = 0; i < N_ITERS; ++i) {
        asm volatile("v_lshlrev_b32 %0, s0, %1\nv_lshlrev_b32 %1, s0, %2\nv_lshlrev_b32 %2, s0, %3\nv_lshlrev_b32 %3, s0, %4\nv_lshlrev_b32 %4, s0, %5\nv_lshlrev_b32 %5, s0, %6\nv_lshlrev_b32 %6, s0, %7\nv_lshlrev_b32 %7, s0, %0" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc", "s0");
    }
    uint64_t r = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
    if ((uint32_t)r == 0x12345678u) out[blockIdx.x] = (uint32_t)r;
}
__global__ __launch_bounds__(1024) void k_v_lshrrev_b32(uint32_t* out, uint32_t seed) {
    uint32_t a0 = seed ^ threadIdx.x, a1 = a0 * 3u, a2 = a0 * 5u, a3 = a0 * 7u, a4 = a0 * 11u, a5 = a0 * 13u, a6 = a0 * 17u, a7 = a0 * 19u;
    for (int i = 0; i < N_ITERS; ++i) {
        asm volatile("v_lshrrev_b32 %0, 3, %1\nv_lshrrev_b32 %1, 3, %2\nv_lshrrev_b32 %2, 3, %3\nv_lshrrev_b32 %3, 3, %4\nv_lshrrev_b32 %4, 3, %5\nv_lshrrev_b32 %5, 3, %6\nv_lshrrev_b32 %6, 3, %7\nv_lshrrev_b32 %7, 3, %0" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc", "s0");
    }
    uint64_t r = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
    if ((uint32_t)r == 0x12345678u) out[blockIdx.x] = (uint32_t)r;
}
__global__ __launch_bounds__(1024) void k_v_or_b32(uint32_t* out, uint32_t seed) {
    uint32_t a0 = seed ^ threadIdx.x, a1 = a0 * 3u, a2 = a0 * 5u, a3 = a0 * 7u, a4 = a0 * 11u, a5 = a0 * 13u, a6 = a0 * 17u, a7 = a0 * 19u;
    for (int i = 0; i < N_ITERS; ++i) {
        asm volatile("v_or_b32 %0, %1, %0\nv_or_b32 %1, %2, %1\nv_or_b32 %2, %3, %2\nv_or_b32 %3, %4, %3\nv_or_b32 %4, %5, %4\nv_or_b32 %5, %6, %5\nv_or_b32 %6, %7, %6\nv_or_b32 %7, %0, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc", "s0");
    }
    uint64_t r = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
    if ((uint32_t)r == 0x12345678u) out[blockIdx.x] = (uint32_t)r;
}
__global__ __launch_bounds__(1024) void k_v_or3_b32(uint32_t* out, uint32_t seed) {
    uint32_t a0 = seed ^ threadIdx.x, a1 = a0 * 3u, a2 = a0 * 5u, a3 = a0 * 7u, a4 = a0 * 11u, a5 = a0 * 13u, a6 = a0 * 17u, a7 = a0 * 19u;
    for (int i = 0; i < N_ITERS; ++i) {
        asm volatile("v_or3_b32 %0, %1, %2, %0\nv_or3_b32 %1, %2, %3, %1\nv_or3_b32 %2, %3, %4, %2\nv_or3_b32 %3, %4, %5, %3\nv_or3_b32 %4, %5, %6, %4\nv_or3_b32 %5, %6, %7, %5\nv_or3_b32 %6, %7, %0, %6\nv_or3_b32 %7, %0, %1, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc", "s0");
    }
    uint64_t r = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
    if ((uint32_t)r == 0x12345678u) out[blockIdx.x] = (uint32_t)r;
}
__global__ __launch_bounds__(1024) void k_v_and_or_b32(uint32_t* out, uint32_t seed) {
    uint32_t a0 = seed ^ threadIdx.x, a1 = a0 * 3u, a2 = a0 * 5u, a3 = a0 * 7u, a4 = a0 * 11u, a5 = a0 * 13u, a6 = a0 * 17u, a7 = a0 * 19u;
    for (int i = 0; i < N_ITERS; ++i) {
        asm volatile("v_and_or_b32 %0, %1, %2, %0\nv_and_or_b32 %1, %2, %3, %1\nv_and_or_b32 %2, %3, %4, %2\nv_and_or_b32 %3, %4, %5, %3\nv_and_or_b32 %4, %5, %6, %4\nv_and_or_b32 %5, %6, %7, %5\nv_and_or_b32 %6, %7, %0, %6\nv_and_or_b32 %7, %0, %1, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc", "s0");
    }
    uint64_t r = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
    if ((uint32_t)r == 0x12345678u) out[blockIdx.x] = (uint32_t)r;
}
__global__ __launch_bounds__(1024) void k_v_bitop3_b32(uint32_t* out, uint32_t seed) {
    uint32_t a0 = seed ^ threadIdx.x, a1 = a0 * 3u, a2 = a0 * 5u, a3 = a0 * 7u, a4 = a0 * 11u, a5 = a0 * 13u, a6 = a0 * 17u, a7 = a0 * 19u;
    for (int i = 0; i < N_ITERS; ++i) {
        asm volatile("v_bitop3_b32 %0, %1, %2, %0 bitop3:0xf8\nv_bitop3_b32 %1, %2, %3, %1 bitop3:0xf8\nv_bitop3_b32 %2, %3, %4, %2 bitop3:0xf8\nv_bitop3_b32 %3, %4, %5, %3 bitop3:0xf8\nv_bitop3_b32 %4, %5, %6, %4 bitop3:0xf8\nv_bitop3_b32 %5, %6, %7, %5 bitop3:0xf8\nv_bitop3_b32 %6, %7, %0, %6 bitop3:0xf8\nv_bitop3_b32 %7, %0, %1, %7 bitop3:0xf8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc", "s0");
    }
    uint64_t r = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
    if ((uint32_t)r == 0x12345678u) out[blockIdx.x] = (uint32_t)r;
}
__global__ __launch_bounds__(1024) void k_v_bcnt_u32_b32(uint32_t* out, uint32_t seed) {
    uint32_t a0 = seed ^ threadIdx.x, a1 = a0 * 3u, a2 = a0 * 5u, a3 = a0 * 7u, a4 = a0 * 11u, a5 = a0 * 13u, a6 = a0 * 17u, a7 = a0 * 19u;
    for (int i = 0; i < N_ITERS; ++i) {
        asm volatile("v_bcnt_u32_b32 %0, %1, %0\nv_bcnt_u32_b32 %1, %2, %1\nv_bcnt_u32_b32 %2, %3, %2\nv_bcnt_u32_b32 %3, %4, %3\nv_bcnt_u32_b32 %4, %5, %4\nv_bcnt_u32_b32 %5, %6, %5\nv_bcnt_u32_b32 %6, %7, %6\nv_bcnt_u32_b32 %7, %0, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc", "s0");
    }
    uint64_t r = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
    if ((uint32_t)r == 0x12345678u) out[blockIdx.x] = (uint32_t)r;
}
__global__ __launch_bounds__(1024) void k_v_alignbit_b32(uint32_t* out, uint32_t seed) {
    uint32_t a0 = seed ^ threadIdx.x, a1 = a0 * 3u, a2 = a0 * 5u, a3 = a0 * 7u, a4 = a0 * 11u, a5 = a0 * 13u, a6 = a0 * 17u, a7 = a0 * 19u;
    for (int i = 0; i < N_ITERS; ++i) {
        asm volatile("v_alignbit_b32 %0, %1, %2, 3\nv_alignbit_b32 %1, %2, %3, 3\nv_alignbit_b32 %2, %3, %4, 3\nv_alignbit_b32 %3, %4, %5, 3\nv_alignbit_b32 %4, %5, %6, 3\nv_alignbit_b32 %5, %6, %7, 3\nv_alignbit_b32 %6, %7, %0, 3\nv_alignbit_b32 %7, %0, %1, 3" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc", "s0");
    }
    uint64_t r = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
    if ((uint32_t)r == 0x12345678u) out[blockIdx.x] = (uint32_t)r;
}
__global__ __launch_bounds__(1024) void k_v_add_u32(uint32_t* out, uint32_t seed) {
    uint32_t a0 = seed ^ threadIdx.x, a1 = a0 * 3u, a2 = a0 * 5u, a3 = a0 * 7u, a4 = a0 * 11u, a5 = a0 * 13u, a6 = a0 * 17u, a7 = a0 * 19u;
    for (int i = 0; i < N_ITERS; ++i) {
        asm volatile("v_add_u32 %0, %1, %0\nv_add_u32 %1, %2, %1\nv_add_u32 %2, %3, %2\nv_add_u32 %3, %4, %3\nv_add_u32 %4, %5, %4\nv_add_u32 %5, %6, %5\nv_add_u32 %6, %7, %6\nv_add_u32 %7, %0, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc", "s0");
    }
    uint64_t r = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
    if ((uint32_t)r == 0x12345678u) out[blockIdx.x] = (uint32_t)r;
}
__global__ __launch_bounds__(1024) void k_v_add3_u32(uint32_t* out, uint32_t seed) {
    uint32_t a0 = seed ^ threadIdx.x, a1 = a0 * 3u, a2 = a0 * 5u, a3 = a0 * 7u, a4 = a0 * 11u, a5 = a0 * 13u, a6 = a0 * 17u, a7 = a0 * 19u;
    for (int i = 0; i < N_ITERS; ++i) {
        asm volatile("v_add3_u32 %0, %1, %2, %0\nv_add3_u32 %1, %2, %3, %1\nv_add3_u32 %2, %3, %4, %2\nv_add3_u32 %3, %4, %5, %3\nv_add3_u32 %4, %5, %6, %4\nv_add3_u32 %5, %6, %7, %5\nv_add3_u32 %6, %7, %0, %6\nv_add3_u32 %7, %0, %1, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc", "s0");
    }
    uint64_t r = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
    if ((uint32_t)r == 0x12345678u) out[blockIdx.x] = (uint32_t)r;
}
__global__ __launch_bounds__(1024) void k_v_lshl_add_u32(uint32_t* out, uint32_t seed) {
    uint32_t a0 = seed ^ threadIdx.x, a1 = a0 * 3u, a2 = a0 * 5u, a3 = a0 * 7u, a4 = a0 * 11u, a5 = a0 * 13u, a6 = a0 * 17u, a7 = a0 * 19u;
    for (int i = 0; i < N_ITERS; ++i) {
        asm volatile("v_lshl_add_u32 %0, %1, 3, %0\nv_lshl_add_u32 %1, %2, 3, %1\nv_lshl_add_u32 %2, %3, 3, %2\nv_lshl_add_u32 %3, %4, 3, %3\nv_lshl_add_u32 %4, %5, 3, %4\nv_lshl_add_u32 %5, %6, 3, %5\nv_lshl_add_u32 %6, %7, 3, %6\nv_lshl_add_u32 %7, %0, 3, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc", "s0");
    }
    uint64_t r = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
    if ((uint32_t)r == 0x12345678u) out[blockIdx.x] = (uint32_t)r;
}
__global__ __launch_bounds__(1024) void k_v_bfe_u32(uint32_t* out, uint32_t seed) {
    uint32_t a0 = seed ^ threadIdx.x, a1 = a0 * 3u, a2 = a0 * 5u, a3 = a0 * 7u, a4 = a0 * 11u, a5 = a0 * 13u, a6 = a0 * 17u, a7 = a0 * 19u;
    for (int i = 0; i < N_ITERS; ++i) {
        asm volatile("v_bfe_u32 %0, %1, 3, 5\nv_bfe_u32 %1, %2, 3, 5\nv_bfe_u32 %2, %3, 3, 5\nv_bfe_u32 %3, %4, 3, 5\nv_bfe_u32 %4, %5, 3, 5\nv_bfe_u32 %5, %6, 3, 5\nv_bfe_u32 %6, %7, 3, 5\nv_bfe_u32 %7, %0, 3, 5" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc", "s0");
    }
    uint64_t r = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
    if ((uint32_t)r == 0x12345678u) out[blockIdx.x] = (uint32_t)r;
}
__global__ __launch_bounds__(1024) void k_v_perm_b32(uint32_t* out, uint32_t seed) {
    uint32_t a0 = seed ^ threadIdx.x, a1 = a0 * 3u, a2 = a0 * 5u, a3 = a0 * 7u, a4 = a0 * 11u, a5 = a0 * 13u, a6 = a0 * 17u, a7 = a0 * 19u;
    for (int i = 0; i < N_ITERS; ++i) {
        asm volatile("v_perm_b32 %0, %1, %2, s0\nv_perm_b32 %1, %2, %3, s0\nv_perm_b32 %2, %3, %4, s0\nv_perm_b32 %3, %4, %5, s0\nv_perm_b32 %4, %5, %6, s0\nv_perm_b32 %5, %6, %7, s0\nv_perm_b32 %6, %7, %0, s0\nv_perm_b32 %7, %0, %1, s0" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc", "s0");
    }
    uint64_t r = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
    if ((uint32_t)r == 0x12345678u) out[blockIdx.x] = (uint32_t)r;
}
__global__ __launch_bounds__(1024) void k_v_cndmask_b32(uint32_t* out, uint32_t seed) {
    uint32_t a0 = seed ^ threadIdx.x, a1 = a0 * 3u, a2 = a0 * 5u, a3 = a0 * 7u, a4 = a0 * 11u, a5 = a0 * 13u, a6 = a0 * 17u, a7 = a0 * 19u;
    for (int i = 0; i < N_ITERS; ++i) {
        asm volatile("v_cndmask_b32 %0, %1, %2, vcc\nv_cndmask_b32 %1, %2, %3, vcc\nv_cndmask_b32 %2, %3, %4, vcc\nv_cndmask_b32 %3, %4, %5, vcc\nv_cndmask_b32 %4, %5, %6, vcc\nv_cndmask_b32 %5, %6, %7, vcc\nv_cndmask_b32 %6, %7, %0, vcc\nv_cndmask_b32 %7, %0, %1, vcc" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc", "s0");
    }
    uint64_t r = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
    if ((uint32_t)r == 0x12345678u) out[blockIdx.x] = (uint32_t)r;
}
__global__ __launch_bounds__(1024) void k_v_mov_b32(uint32_t* out, uint32_t seed) {
    uint32_t a0 = seed ^ threadIdx.x, a1 = a0 * 3u, a2 = a0 * 5u, a3 = a0 * 7u, a4 = a0 * 11u, a5 = a0 * 13u, a6 = a0 * 17u, a7 = a0 * 19u;
    for (int i = 0; i < N_ITERS; ++i) {
        asm volatile("v_mov_b32 %0, %1\nv_mov_b32 %1, %2\nv_mov_b32 %2, %3\nv_mov_b32 %3, %4\nv_mov_b32 %4, %5\nv_mov_b32 %5, %6\nv_mov_b32 %6, %7\nv_mov_b32 %7, %0" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc", "s0");
    }
    uint64_t r = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
    if ((uint32_t)r == 0x12345678u) out[blockIdx.x] = (uint32_t)r;
}
__global__ __launch_bounds__(1024) void k_v_not_b32(uint32_t* out, uint32_t seed) {
    uint32_t a0 = seed ^ threadIdx.x, a1 = a0 * 3u, a2 = a0 * 5u, a3 = a0 * 7u, a4 = a0 * 11u, a5 = a0 * 13u, a6 = a0 * 17u, a7 = a0 * 19u;
    for (int i = 0; i < N_ITERS; ++i) {
        asm volatile("v_not_b32 %0, %1\nv_not_b32 %1, %2\nv_not_b32 %2, %3\nv_not_b32 %3, %4\nv_not_b32 %4, %5\nv_not_b32 %5, %6\nv_not_b32 %6, %7\nv_not_b32 %7, %0" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc", "s0");
    }
    uint64_t r = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
    if ((uint32_t)r == 0x12345678u) out[blockIdx.x] = (uint32_t)r;
}
__global__ __launch_bounds__(1024) void k_v_pk_lshlrev_b16(uint32_t* out, uint32_t seed) {
    uint32_t a0 = seed ^ threadIdx.x, a1 = a0 * 3u, a2 = a0 * 5u, a3 = a0 * 7u, a4 = a0 * 11u, a5 = a0 * 13u, a6 = a0 * 17u, a7 = a0 * 19u;
    for (int i = 0; i < N_ITERS; ++i) {
        asm volatile("v_pk_lshlrev_b16 %0, 3, %1\nv_pk_lshlrev_b16 %1, 3, %2\nv_pk_lshlrev_b16 %2, 3, %3\nv_pk_lshlrev_b16 %3, 3, %4\nv_pk_lshlrev_b16 %4, 3, %5\nv_pk_lshlrev_b16 %5, 3, %6\nv_pk_lshlrev_b16 %6, 3, %7\nv_pk_lshlrev_b16 %7, 3, %0" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc", "s0");
    }
    uint64_t r = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
    if ((uint32_t)r == 0x12345678u) out[blockIdx.x] = (uint32_t)r;
}
__global__ __launch_bounds__(1024) void k_v_mul_lo_u32(uint32_t* out, uint32_t seed) {
    uint32_t a0 = seed ^ threadIdx.x, a1 = a0 * 3u, a2 = a0 * 5u, a3 = a0 * 7u, a4 = a0 * 11u, a5 = a0 * 13u, a6 = a0 * 17u, a7 = a0 * 19u;
    for (int i = 0; i < N_ITERS; ++i) {
        asm volatile("v_mul_lo_u32 %0, %1, %2\nv_mul_lo_u32 %1, %2, %3\nv_mul_lo_u32 %2, %3, %4\nv_mul_lo_u32 %3, %4, %5\nv_mul_lo_u32 %4, %5, %6\nv_mul_lo_u32 %5, %6, %7\nv_mul_lo_u32 %6, %7, %0\nv_mul_lo_u32 %7, %0, %1" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc", "s0");
    }
    uint64_t r = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
    if ((uint32_t)r == 0x12345678u) out[blockIdx.x] = (uint32_t)r;
}
__global__ __launch_bounds__(1024) void k_v_mad_u32_u24(uint32_t* out, uint32_t seed) {
    uint32_t a0 = seed ^ threadIdx.x, a1 = a0 * 3u, a2 = a0 * 5u, a3 = a0 * 7u, a4 = a0 * 11u, a5 = a0 * 13u, a6 = a0 * 17u, a7 = a0 * 19u;
    for (int i = 0; i < N_ITERS; ++i) {
        asm volatile("v_mad_u32_u24 %0, %1, %2, %0\nv_mad_u32_u24 %1, %2, %3, %1\nv_mad_u32_u24 %2, %3, %4, %2\nv_mad_u32_u24 %3, %4, %5, %3\nv_mad_u32_u24 %4, %5, %6, %4\nv_mad_u32_u24 %5, %6, %7, %5\nv_mad_u32_u24 %6, %7, %0, %6\nv_mad_u32_u24 %7, %0, %1, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc", "s0");
    }
    uint64_t r = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
    if ((uint32_t)r == 0x12345678u) out[blockIdx.x] = (uint32_t)r;
}
__global__ __launch_bounds__(1024) void k_v_xor_b32(uint32_t* out, uint32_t seed) {
    uint32_t a0 = seed ^ threadIdx.x, a1 = a0 * 3u, a2 = a0 * 5u, a3 = a0 * 7u, a4 = a0 * 11u, a5 = a0 * 13u, a6 = a0 * 17u, a7 = a0 * 19u;
    for (int i = 0; i < N_ITERS; ++i) {
        asm volatile("v_xor_b32 %0, %1, %0\nv_xor_b32 %1, %2, %1\nv_xor_b32 %2, %3, %2\nv_xor_b32 %3, %4, %3\nv_xor_b32 %4, %5, %4\nv_xor_b32 %5, %6, %5\nv_xor_b32 %6, %7, %6\nv_xor_b32 %7, %0, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc", "s0");
    }
    uint64_t r = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
    if ((uint32_t)r == 0x12345678u) out[blockIdx.x] = (uint32_t)r;
}
__global__ __launch_bounds__(1024) void k_v_bfi_b32(uint32_t* out, uint32_t seed) {
    uint32_t a0 = seed ^ threadIdx.x, a1 = a0 * 3u, a2 = a0 * 5u, a3 = a0 * 7u, a4 = a0 * 11u, a5 = a0 * 13u, a6 = a0 * 17u, a7 = a0 * 19u;
    for (int i = 0; i < N_ITERS; ++i) {
        asm volatile("v_bfi_b32 %0, %1, %2, %0\nv_bfi_b32 %1, %2, %3, %1\nv_bfi_b32 %2, %3, %4, %2\nv_bfi_b32 %3, %4, %5, %3\nv_bfi_b32 %4, %5, %6, %4\nv_bfi_b32 %5, %6, %7, %5\nv_bfi_b32 %6, %7, %0, %6\nv_bfi_b32 %7, %0, %1, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc", "s0");
    }
    uint64_t r = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
    if ((uint32_t)r == 0x12345678u) out[blockIdx.x] = (uint32_t)r;
}
__global__ __launch_bounds__(1024) void k_v_lshlrev_b64(uint32_t* out, uint32_t seed) {
    uint64_t a0 = seed ^ threadIdx.x, a1 = a0 * 3u, a2 = a0 * 5u, a3 = a0 * 7u, a4 = a0 * 11u, a5 = a0 * 13u, a6 = a0 * 17u, a7 = a0 * 19u;
    for (int i = 0; i < N_ITERS; ++i) {
        asm volatile("v_lshlrev_b64 %0, 3, %1\nv_lshlrev_b64 %1, 3, %2\nv_lshlrev_b64 %2, 3, %3\nv_lshlrev_b64 %3, 3, %4\nv_lshlrev_b64 %4, 3, %5\nv_lshlrev_b64 %5, 3, %6\nv_lshlrev_b64 %6, 3, %7\nv_lshlrev_b64 %7, 3, %0" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc", "s0");
    }
    uint64_t r = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
    if ((uint32_t)r == 0x12345678u) out[blockIdx.x] = (uint32_t)r;
}
__global__ __launch_bounds__(1024) void k_v_lshl_add_u64(uint32_t* out, uint32_t seed) {
    uint64_t a0 = seed ^ threadIdx.x, a1 = a0 * 3u, a2 = a0 * 5u, a3 = a0 * 7u, a4 = a0 * 11u, a5 = a0 * 13u, a6 = a0 * 17u, a7 = a0 * 19u;
    for (int i = 0; i < N_ITERS; ++i) {
        asm volatile("v_lshl_add_u64 %0, %1, 3, %0\nv_lshl_add_u64 %1, %2, 3, %1\nv_lshl_add_u64 %2, %3, 3, %2\nv_lshl_add_u64 %3, %4, 3, %3\nv_lshl_add_u64 %4, %5, 3, %4\nv_lshl_add_u64 %5, %6, 3, %5\nv_lshl_add_u64 %6, %7, 3, %6\nv_lshl_add_u64 %7, %0, 3, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc", "s0");
    }
    uint64_t r = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
    if ((uint32_t)r == 0x12345678u) out[blockIdx.x] = (uint32_t)r;
}
__global__ __launch_bounds__(1024) void k_v_pk_mov_b32(uint32_t* out, uint32_t seed) {
    uint64_t a0 = seed ^ threadIdx.x, a1 = a0 * 3u, a2 = a0 * 5u, a3 = a0 * 7u, a4 = a0 * 11u, a5 = a0 * 13u, a6 = a0 * 17u, a7 = a0 * 19u;
    for (int i = 0; i < N_ITERS; ++i) {
        asm volatile("v_pk_mov_b32 %0, %1, %0 op_sel:[0,1]\nv_pk_mov_b32 %1, %2, %1 op_sel:[0,1]\nv_pk_mov_b32 %2, %3, %2 op_sel:[0,1]\nv_pk_mov_b32 %3, %4, %3 op_sel:[0,1]\nv_pk_mov_b32 %4, %5, %4 op_sel:[0,1]\nv_pk_mov_b32 %5, %6, %5 op_sel:[0,1]\nv_pk_mov_b32 %6, %7, %6 op_sel:[0,1]\nv_pk_mov_b32 %7, %0, %7 op_sel:[0,1]" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc", "s0");
    }
    uint64_t r = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
    if ((uint32_t)r == 0x12345678u) out[blockIdx.x] = (uint32_t)r;
}

__global__ __launch_bounds__(1024) void k_cnd_e64(uint32_t* out, uint32_t seed) {
    uint32_t a0 = seed ^ threadIdx.x, a1 = a0 * 3u, a2 = a0 * 5u, a3 = a0 * 7u, a4 = a0 * 11u, a5 = a0 * 13u, a6 = a0 * 17u, a7 = a0 * 19u;
    uint64_t m = __builtin_amdgcn_ballot_w64(threadIdx.x & 1);
    for (int i = 0; i < N_ITERS; ++i) {
        asm volatile("v_cndmask_b32_e64 %0, %1, %2, %8\nv_cndmask_b32_e64 %1, %2, %3, %8\nv_cndmask_b32_e64 %2, %3, %4, %8\nv_cndmask_b32_e64 %3, %4, %5, %8\nv_cndmask_b32_e64 %4, %5, %6, %8\nv_cndmask_b32_e64 %5, %6, %7, %8\nv_cndmask_b32_e64 %6, %7, %0, %8\nv_cndmask_b32_e64 %7, %0, %1, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "s"(m));
    }
    uint64_t r = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
    if ((uint32_t)r == 0x12345678u) out[blockIdx.x] = (uint32_t)r;
}
__global__ __launch_bounds__(1024) void k_cmp_cnd(uint32_t* out, uint32_t seed) {
    uint32_t a0 = seed ^ threadIdx.x, a1 = a0 * 3u, a2 = a0 * 5u, a3 = a0 * 7u, a4 = a0 * 11u, a5 = a0 * 13u, a6 = a0 * 17u, a7 = a0 * 19u;
    for (int i = 0; i < N_ITERS; ++i) {
        // the select pattern the compiler emits for c ? x : y with a per-lane condition
        a0 = (a1 > a2) ? a3 : a4; a1 = (a2 > a3) ? a4 : a5; a2 = (a3 > a4) ? a5 : a6; a3 = (a4 > a5) ? a6 : a7;
        a4 = (a5 > a6) ? a7 : a0; a5 = (a6 > a7) ? a0 : a1; a6 = (a7 > a0) ? a1 : a2; a7 = (a0 > a1) ? a2 : a3;
    }
    uint64_t r = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
    if ((uint32_t)r == 0x12345678u) out[blockIdx.x] = (uint32_t)r;
}
__global__ __launch_bounds__(1024) void k_cmp_only(uint32_t* out, uint32_t seed) {
    uint32_t a0 = seed ^ threadIdx.x, a1 = a0 * 3u;
    uint64_t acc = 0;
    for (int i = 0; i < N_ITERS; ++i) {
        uint64_t m0, m1, m2, m3, m4, m5, m6, m7;
        asm volatile("v_cmp_gt_u32_e64 %0, %8, %9\nv_cmp_gt_u32_e64 %1, %9, %8\nv_cmp_gt_u32_e64 %2, %8, %9\nv_cmp_gt_u32_e64 %3, %9, %8\nv_cmp_gt_u32_e64 %4, %8, %9\nv_cmp_gt_u32_e64 %5, %9, %8\nv_cmp_gt_u32_e64 %6, %8, %9\nv_cmp_gt_u32_e64 %7, %9, %8" : "=s"(m0), "=s"(m1), "=s"(m2), "=s"(m3), "=s"(m4), "=s"(m5), "=s"(m6), "=s"(m7) : "v"(a0), "v"(a1));
        acc ^= m0 ^ m1 ^ m2 ^ m3 ^ m4 ^ m5 ^ m6 ^ m7;
    }
    if ((uint32_t)acc == 0x12345678u) out[blockIdx.x] = (uint32_t)acc;
}

// dependent chains: every instruction reads the previous one's result
#define DEP_KERNEL(NAME, INSN)                                                                    \
__global__ __launch_bounds__(1024) void NAME(uint32_t* out, uint32_t seed) {                     \
    uint32_t a0 = seed ^ threadIdx.x, a1 = a0 * 3u, a2 = a0 * 5u;                                \
    for (int i = 0; i < N_ITERS; ++i) {                                                            \
        asm volatile(INSN "\n" INSN "\n" INSN "\n" INSN "\n" INSN "\n" INSN "\n" INSN "\n" INSN \
                     : "+v"(a0) : "v"(a1), "v"(a2));                                               \
    }                                                                                              \
    if (a0 == 0x12345678u) out[blockIdx.x] = a0;                                                   \
}
DEP_KERNEL(k_dep_or, "v_or_b32 %0, %1, %0")
DEP_KERNEL(k_dep_lshr, "v_lshrrev_b32 %0, 1, %0")
DEP_KERNEL(k_dep_bitop3, "v_bitop3_b32 %0, %1, %2, %0 bitop3:0xfe")
DEP_KERNEL(k_dep_lshl_or, "v_lshl_or_b32 %0, %1, 3, %0")
DEP_KERNEL(k_dep_bcnt, "v_bcnt_u32_b32 %0, %1, %0")

// realistic stencil mixes (8 statements per iteration)
__global__ __launch_bounds__(1024) void k_mix_lshr_s(uint32_t* out, uint32_t seed) {
    uint32_t a0 = seed ^ threadIdx.x, a1 = a0 * 3u, a2 = a0 * 5u, a3 = a0 * 7u, a4 = a0 * 11u, a5 = a0 * 13u, a6 = a0 * 17u, a7 = a0 * 19u;
    const uint32_t sh = seed & 7u;
    for (int i = 0; i < N_ITERS; ++i) {
        asm volatile("v_lshrrev_b32 %0, %8, %1\nv_lshrrev_b32 %1, %8, %2\nv_lshrrev_b32 %2, %8, %3\nv_lshrrev_b32 %3, %8, %4\n"
                     "v_lshrrev_b32 %4, %8, %5\nv_lshrrev_b32 %5, %8, %6\nv_lshrrev_b32 %6, %8, %7\nv_lshrrev_b32 %7, %8, %0"
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "s"(sh));
    }
    uint32_t r = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
    if (r == 0x12345678u) out[blockIdx.x] = r;
}
// 3 lshrrev(s) + 2 bitop3 + 1 bcnt + 2 lshrrev  (8 ops, one slow)
__global__ __launch_bounds__(1024) void k_mix_sten(uint32_t* out, uint32_t seed) {
    uint32_t a0 = seed ^ threadIdx.x, a1 = a0 * 3u, a2 = a0 * 5u, a3 = a0 * 7u, a4 = a0 * 11u, a5 = a0 * 13u, a6 = a0 * 17u, a7 = a0 * 19u;
    const uint32_t sh = seed & 7u;
    for (int i = 0; i < N_ITERS; ++i) {
        asm volatile("v_lshrrev_b32 %0, %8, %1\nv_lshrrev_b32 %1, %8, %2\nv_bitop3_b32 %2, %3, %0, %1 bitop3:0xfe\nv_lshrrev_b32 %3, %8, %4\n"
                     "v_lshrrev_b32 %4, %8, %5\nv_bitop3_b32 %5, %6, %3, %4 bitop3:0x54\nv_bcnt_u32_b32 %6, %5, %6\nv_lshrrev_b32 %7, %8, %0"
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "s"(sh));
    }
    uint32_t r = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
    if (r == 0x12345678u) out[blockIdx.x] = r;
}

#define MIX_KERNEL(NAME, BODY, CONS)                                                               \
__global__ __launch_bounds__(1024) void NAME(uint32_t* out, uint32_t seed) {                     \
    uint32_t a0 = seed ^ threadIdx.x, a1 = a0 * 3u, a2 = a0 * 5u, a3 = a0 * 7u, a4 = a0 * 11u,   \
             a5 = a0 * 13u, a6 = a0 * 17u, a7 = a0 * 19u;                                         \
    uint32_t sh = seed & 7u;                                                                      \
    uint32_t vsh = __builtin_amdgcn_readfirstlane(sh) + (threadIdx.x >> 10);                      \
    for (int i = 0; i < N_ITERS; ++i) {                                                            \
        asm volatile(BODY : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), \
                     "+v"(a7) : CONS);                                                             \
    }                                                                                              \
    uint32_t r = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;                                            \
    if (r == 0x12345678u) out[blockIdx.x] = r;                                                     \
}
#define R8(I) I(0,1) I(1,2) I(2,3) I(3,4) I(4,5) I(5,6) I(6,7) I(7,0)
#define LSHR_V(d, a) "v_lshrrev_b32 %" #d ", %8, %" #a "\n"
#define OR_S(d, a) "v_or_b32 %" #d ", %8, %" #a "\n"
#define BITOP3_S(d, a) "v_bitop3_b32 %" #d ", %" #a ", %8, %" #d " bitop3:0xfe\n"
#define ALIGN_V(d, a) "v_alignbit_b32 %" #d ", %" #a ", %" #d ", %8\n"
MIX_KERNEL(k_lshr_v, R8(LSHR_V), "v"(vsh))
MIX_KERNEL(k_or_s, R8(OR_S), "s"(sh))
MIX_KERNEL(k_bitop3_s, R8(BITOP3_S), "s"(sh))
MIX_KERNEL(k_lshr_inl, "v_lshrrev_b32 %0, 3, %1\nv_lshrrev_b32 %1, 3, %2\nv_lshrrev_b32 %2, 3, %3\nv_lshrrev_b32 %3, 3, %4\nv_lshrrev_b32 %4, 3, %5\nv_lshrrev_b32 %5, 3, %6\nv_lshrrev_b32 %6, 3, %7\nv_lshrrev_b32 %7, 3, %0", "v"(vsh))

typedef void (*kfn)(uint32_t*, uint32_t);
static void run(const char* name, kfn f, uint32_t* d, int num_cu) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    printf("%-18s", name);
    for (int wps = 1; wps <= 4; ++wps) {
        const int threads = 64 * 4 * wps;
        hipLaunchKernelGGL(f, dim3(num_cu), dim3(threads), 0, 0, d, 1u);
        (void)hipEventRecord(e0);
        for (int k = 0; k < 5; ++k) hipLaunchKernelGGL(f, dim3(num_cu), dim3(threads), 0, 0, d, 1u);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms; (void)hipEventElapsedTime(&ms, e0, e1);
        const double ns = ms / 5 * 1e6 / ((double)wps * N_ITERS * 8.0);
        printf("  w%d: %.2f cyc", wps, ns * 2.4);
    }
    printf("\n");
}
int main() {
    hipDeviceProp_t p; (void)hipGetDeviceProperties(&p, 0);
    uint32_t* d; (void)hipMalloc(&d, 4096 * 4);
    printf("cycles per wave64 instruction per SIMD at 2.4 GHz (w = waves per SIMD)\n");

    run("v_lshl_or_b32", k_v_lshl_or_b32, d, p.multiProcessorCount);
    run("v_lshlrev_b32", k_v_lshlrev_b32, d, p.multiProcessorCount);
    run("v_lshlrev_b32_s", k_v_lshlrev_b32_s, d, p.multiProcessorCount);
    run("v_lshrrev_b32", k_v_lshrrev_b32, d, p.multiProcessorCount);
    run("v_or_b32", k_v_or_b32, d, p.multiProcessorCount);
    run("v_or3_b32", k_v_or3_b32, d, p.multiProcessorCount);
    run("v_and_or_b32", k_v_and_or_b32, d, p.multiProcessorCount);
    run("v_bitop3_b32", k_v_bitop3_b32, d, p.multiProcessorCount);
    run("v_bcnt_u32_b32", k_v_bcnt_u32_b32, d, p.multiProcessorCount);
    run("v_alignbit_b32", k_v_alignbit_b32, d, p.multiProcessorCount);
    run("v_add_u32", k_v_add_u32, d, p.multiProcessorCount);
    run("v_add3_u32", k_v_add3_u32, d, p.multiProcessorCount);
    run("v_lshl_add_u32", k_v_lshl_add_u32, d, p.multiProcessorCount);
    run("v_bfe_u32", k_v_bfe_u32, d, p.multiProcessorCount);
    run("v_perm_b32", k_v_perm_b32, d, p.multiProcessorCount);
    run("v_cndmask_b32", k_v_cndmask_b32, d, p.multiProcessorCount);
    run("v_mov_b32", k_v_mov_b32, d, p.multiProcessorCount);
    run("v_not_b32", k_v_not_b32, d, p.multiProcessorCount);
    run("v_pk_lshlrev_b16", k_v_pk_lshlrev_b16, d, p.multiProcessorCount);
    run("v_mul_lo_u32", k_v_mul_lo_u32, d, p.multiProcessorCount);
    run("v_mad_u32_u24", k_v_mad_u32_u24, d, p.multiProcessorCount);
    run("v_xor_b32", k_v_xor_b32, d, p.multiProcessorCount);
    run("v_bfi_b32", k_v_bfi_b32, d, p.multiProcessorCount);
    run("v_lshlrev_b64", k_v_lshlrev_b64, d, p.multiProcessorCount);
    run("v_lshl_add_u64", k_v_lshl_add_u64, d, p.multiProcessorCount);
    run("v_pk_mov_b32", k_v_pk_mov_b32, d, p.multiProcessorCount);
    run("v_cndmask_e64", k_cnd_e64, d, p.multiProcessorCount);
    run("cmp+cndmask(C)", k_cmp_cnd, d, p.multiProcessorCount);
    run("v_cmp_e64", k_cmp_only, d, p.multiProcessorCount);
    run("dep v_or", k_dep_or, d, p.multiProcessorCount);
    run("dep v_lshrrev", k_dep_lshr, d, p.multiProcessorCount);
    run("dep v_bitop3", k_dep_bitop3, d, p.multiProcessorCount);
    run("dep v_lshl_or", k_dep_lshl_or, d, p.multiProcessorCount);
    run("dep v_bcnt", k_dep_bcnt, d, p.multiProcessorCount);
    run("lshrrev(s)", k_mix_lshr_s, d, p.multiProcessorCount);
    run("stencil mix 7f+1s", k_mix_sten, d, p.multiProcessorCount);
    run("lshrrev(v)", k_lshr_v, d, p.multiProcessorCount);
    run("lshrrev(inline)", k_lshr_inl, d, p.multiProcessorCount);
    run("or(s)", k_or_s, d, p.multiProcessorCount);
    run("bitop3(s)", k_bitop3_s, d, p.multiProcessorCount);
    return 0;
}
