#!/usr/bin/env python3
"""Emit tools/valu_probe3.hip: does a v_bcnt-free stream dual-issue when the popcounts
are clustered at the end of each orientation?  (carry-save movegen.)

Each kernel loops over one asm block of F fast ops (v_lshrrev_b32 by a VGPR amount and
v_bitop3_b32, VGPR operands only) plus S v_bcnt_u32_b32, either clustered after the
fast ops or spread evenly; prints cycles per wave64 instruction per SIMD for 1..4
waves per SIMD."""
import os

HERE = os.path.dirname(os.path.abspath(__file__))


def body(F, S, spread):
    ops = []
    for i in range(F):
        d, a, b = i % 8, (i + 3) % 8, (i + 5) % 8
        if i % 2 == 0:
            ops.append(f"v_lshrrev_b32 %{d}, %8, %{a}")
        else:
            ops.append(f"v_bitop3_b32 %{d}, %{a}, %{b}, %{d} bitop3:0x96")
    slow = [f"v_bcnt_u32_b32 %{i % 8}, %{(i + 2) % 8}, %{i % 8}" for i in range(S)]
    if spread and S:
        step = F // S
        out = []
        for i, op in enumerate(ops):
            out.append(op)
            if (i + 1) % step == 0 and slow:
                out.append(slow.pop(0))
        out += slow
        ops = out
    else:
        ops = ops + slow
    return "\\n".join(ops)


CASES = [("fast96", 96, 0, False), ("fast96+4bcnt_end", 96, 4, False), ("fast192+8bcnt_end", 192, 8, False),
         ("fast384+16bcnt_end", 384, 16, False), ("fast96+4bcnt_spread", 96, 4, True),
         ("fast192+17bcnt_end", 192, 17, False), ("fast88+8bcnt_spread", 88, 8, True)]

src = ['#include <hip/hip_runtime.h>', '#include <stdint.h>', '#include <stdio.h>', '#define N_ITERS 4096', '']
for name, F, S, spread in CASES:
    k = "k_" + name.replace("+", "_")
    src.append(f'''__global__ __launch_bounds__(1024) void {k}(uint32_t* out, uint32_t seed) {{
    uint32_t a0 = seed ^ threadIdx.x, a1 = a0 * 3u, a2 = a0 * 5u, a3 = a0 * 7u, a4 = a0 * 11u, a5 = a0 * 13u, a6 = a0 * 17u, a7 = a0 * 19u;
    uint32_t vsh = __builtin_amdgcn_readfirstlane(seed & 7u) + (threadIdx.x >> 10);
    for (int i = 0; i < N_ITERS / 16; ++i) {{
        asm volatile("{body(F, S, spread)}"
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(vsh));
    }}
    uint32_t r = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
    if (r == 0x12345678u) out[blockIdx.x] = r;
}}
''')
src.append('''typedef void (*kfn)(uint32_t*, uint32_t);
static void run(const char* name, kfn f, int ops, uint32_t* d, int num_cu) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    printf("%-22s", name);
    for (int wps = 1; wps <= 4; ++wps) {
        const int threads = 64 * 4 * wps;
        hipLaunchKernelGGL(f, dim3(num_cu), dim3(threads), 0, 0, d, 1u);
        (void)hipEventRecord(e0);
        for (int k = 0; k < 5; ++k) hipLaunchKernelGGL(f, dim3(num_cu), dim3(threads), 0, 0, d, 1u);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms; (void)hipEventElapsedTime(&ms, e0, e1);
        const double ns = ms / 5 * 1e6 / ((double)wps * (N_ITERS / 16) * ops);
        printf("  w%d: %.2f cyc", wps, ns * 2.4);
    }
    printf("\\n");
}
int main() {
    hipDeviceProp_t p; (void)hipGetDeviceProperties(&p, 0);
    uint32_t* d; (void)hipMalloc(&d, 4096 * 4);
    printf("cycles per wave64 instruction per SIMD at 2.4 GHz (w = waves per SIMD)\\n");''')
for name, F, S, spread in CASES:
    k = "k_" + name.replace("+", "_")
    src.append(f'    run("{name}", {k}, {F + S}, d, p.multiProcessorCount);')
src.append('    return 0;\n}\n')
open(os.path.join(HERE, "valu_probe3.hip"), "w").write("\n".join(src))
