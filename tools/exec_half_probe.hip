// Does a wave64 VALU instruction cost less when one 32-lane half of EXEC is zero?
// (GPU box; diagnostic only.)  One wave per SIMD runs the same dependent-free VALU
// stream under four masks: all 64 lanes, lanes 0..31, even lanes, lanes 0..15.  Prints
// shader-clock cycles per instruction for each.  Build:
//   hipcc --offload-arch=gfx950 -O3 -o tools/_bin/exec_half_probe tools/exec_half_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>

#define N_ITER 4096

__global__ void probe(int mode, unsigned long long* out, unsigned* sink) {
    const int lane = threadIdx.x & 63;
    bool on = true;
    if (mode == 1) on = lane < 32;
    if (mode == 2) on = (lane & 1) == 0;
    if (mode == 3) on = lane < 16;
    unsigned a = lane * 3u + 1u, b = lane ^ 0x55u, c = lane + 7u, d = lane * 11u, e = lane + 13u, f = lane * 5u;
    unsigned long long t0 = 0, t1 = 0;
    if (on) {
        t0 = clock64();
#pragma unroll 1
        for (int i = 0; i < N_ITER; ++i) {
            // 6 independent chains of fast ops (bitop3 / xor / add)
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                a = __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
                b = __builtin_amdgcn_bitop3_b32(b, c, d, 0x96);
                c = __builtin_amdgcn_bitop3_b32(c, d, e, 0x96);
                d = __builtin_amdgcn_bitop3_b32(d, e, f, 0x96);
                e = __builtin_amdgcn_bitop3_b32(e, f, a, 0x96);
                f = __builtin_amdgcn_bitop3_b32(f, a, b, 0x96);
            }
        }
        t1 = clock64();
    }
    if (on) sink[blockIdx.x * 64 + lane] = a ^ b ^ c ^ d ^ e ^ f;
    if (lane == 0 || (mode == 2 && lane == 0)) out[blockIdx.x] = t1 - t0;
}

int main() {
    const int blocks = 256 * 4;  // one wave per SIMD
    unsigned long long* d_out;
    unsigned* d_sink;
    hipMalloc(&d_out, blocks * sizeof(unsigned long long));
    hipMalloc(&d_sink, blocks * 64 * sizeof(unsigned));
    const char* names[4] = {"all 64 lanes", "lanes 0..31", "even lanes", "lanes 0..15"};
    for (int mode = 0; mode < 4; ++mode) {
        for (int rep = 0; rep < 2; ++rep) {
            hipLaunchKernelGGL(probe, dim3(blocks), dim3(64), 0, 0, mode, d_out, d_sink);
            hipDeviceSynchronize();
        }
        unsigned long long h[blocks];
        hipMemcpy(h, d_out, sizeof h, hipMemcpyDeviceToHost);
        double s = 0;
        for (int i = 0; i < blocks; ++i) s += (double)h[i];
        const double insts = (double)N_ITER * 8 * 6;
        printf("{\"mask\": \"%s\", \"cycles_per_valu_inst\": %.3f}\n", names[mode], s / blocks / insts);
    }
    hipFree(d_out);
    hipFree(d_sink);
    return 0;
}
