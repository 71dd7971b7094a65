// Issue-rate microbenchmark (dev tool): how many SALU / VALU / mixed instructions per cycle a
// CU sustains with W waves per SIMD on gfx950.  Each wave runs ITER iterations of a 32-instruction
// block of independent ops; the host reports instructions per cycle per SIMD and per CU.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define ITER 4096
#define S8(op) op " s[20:21], s[22:23]\n" op " s[24:25], s[26:27]\n" op " s[28:29], s[30:31]\n" op " s[32:33], s[34:35]\n" \
               op " s[36:37], s[38:39]\n" op " s[40:41], s[42:43]\n" op " s[44:45], s[46:47]\n" op " s[48:49], s[50:51]\n"
#define V8(op) op " v10, v11, v12\n" op " v13, v14, v15\n" op " v16, v17, v18\n" op " v19, v20, v21\n" \
               op " v22, v23, v24\n" op " v25, v26, v27\n" op " v28, v29, v30\n" op " v31, v32, v33\n"

template <int KIND>
__global__ __launch_bounds__(64) void k(unsigned long long* out) {
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < ITER; ++i) {
        if (KIND == 0) asm volatile(S8("s_not_b64") S8("s_not_b64") S8("s_not_b64") S8("s_not_b64") ::: "memory",
                                    "s20","s21","s22","s23","s24","s25","s26","s27","s28","s29","s30","s31","s32","s33","s34","s35",
                                    "s36","s37","s38","s39","s40","s41","s42","s43","s44","s45","s46","s47","s48","s49","s50","s51");
        if (KIND == 1) asm volatile(V8("v_xor_b32") V8("v_xor_b32") V8("v_xor_b32") V8("v_xor_b32") ::: "memory",
                                    "v10","v11","v12","v13","v14","v15","v16","v17","v18","v19","v20","v21","v22","v23","v24","v25",
                                    "v26","v27","v28","v29","v30","v31","v32","v33");
        if (KIND == 2) asm volatile(S8("s_not_b64") V8("v_xor_b32") S8("s_not_b64") V8("v_xor_b32") ::: "memory",
                                    "s20","s21","s22","s23","s24","s25","s26","s27","s28","s29","s30","s31","s32","s33","s34","s35",
                                    "s36","s37","s38","s39","s40","s41","s42","s43","s44","s45","s46","s47","s48","s49","s50","s51",
                                    "v10","v11","v12","v13","v14","v15","v16","v17","v18","v19","v20","v21","v22","v23","v24","v25",
                                    "v26","v27","v28","v29","v30","v31","v32","v33");
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) atomicAdd(&out[0], t1 - t0), atomicAdd(&out[1], 1ull);
}

int main() {
    setvbuf(stdout, NULL, _IONBF, 0);
    printf("start\n");
    unsigned long long* d; hipMalloc(&d, 16);
    const char* names[3] = {"salu", "valu", "mix(1:1)"};
    for (int kind = 0; kind < 3; ++kind)
        for (int w = 1; w <= 8; w *= 2) {
            int blocks = 256 * 4 * w;
            hipMemset(d, 0, 16);
            hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
            auto launch = [&]() {
                if (kind == 0) k<0><<<blocks, 64>>>(d);
                if (kind == 1) k<1><<<blocks, 64>>>(d);
                if (kind == 2) k<2><<<blocks, 64>>>(d);
            };
            printf("launch %d %d\n", kind, w);
            launch(); hipError_t e = hipDeviceSynchronize(); printf("sync %s\n", hipGetErrorString(e)); hipMemset(d, 0, 16);
            hipEventRecord(a); launch(); hipEventRecord(b); hipEventSynchronize(b);
            float ms; hipEventElapsedTime(&ms, a, b);
            unsigned long long h[2]; hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
            double cyc = (double)h[0] / h[1];                 // cycles per wave (s_memtime ticks)
            double insts = 32.0 * ITER;
            // per SIMD: w waves each issuing insts in cyc cycles (all resident at once)
            printf("%-9s waves/SIMD %d: %.0f cycles per wave, %.3f instr/cycle/wave, %.3f instr/cycle/SIMD, wall %.3f ms\n",
                   names[kind], w, cyc, insts / cyc, w * insts / cyc, ms);
        }
    return 0;
}
