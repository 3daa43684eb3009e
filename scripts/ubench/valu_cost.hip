// Issue cost of the vector instructions the render loop is made of, on gfx950.
//
// Each lane runs CHAINS independent chains of one instruction.  The grid holds exactly
// W waves per SIMD (W = 1, 2, 4, 8; cus * W workgroups of 4 waves, all resident at once),
// so in the s_memtime interval a wave spends in its loop, its SIMD issues W * insts
// wave-instructions:
//     cycles per wave-instruction per SIMD = d(s_memtime) / (W * insts)
// s_memtime counts shader-clock cycles; s_memrealtime a constant 100 MHz, so
//     clock = d(s_memtime) / d(s_memrealtime) * 100 MHz
// is the clock the chip actually held in the loop (DVFS lowers it under load), and
//     wave-instructions per second per SIMD = clock / cycles
// the rate the render kernel's SQ_INSTS_VALU / (1024 SIMDs x kernel time) is compared with.
// Build: hipcc --offload-arch=gfx950 -O3 -o valu_cost valu_cost.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <algorithm>

typedef float f32x2 __attribute__((ext_vector_type(2)));
constexpr int ITERS = 65536, CHAINS = 8, UNROLL = 4;

#define DEF_OP(NAME, T, INIT, BODY)                                                           \
    struct NAME {                                                                           \
        using type = T;                                                                     \
        static __device__ __forceinline__ T init(uint32_t i) { return INIT; }               \
        static __device__ __forceinline__ void step(T& a, T b) { BODY; }                    \
        static constexpr const char* name = #NAME;                                          \
    };

DEF_OP(v_xor_b32, uint32_t, i * 2654435761u, asm volatile("v_xor_b32 %0, %1, %0" : "+v"(a) : "v"(b)))
DEF_OP(v_add_f32, float, 1.0f + i * 1e-7f, asm volatile("v_add_f32 %0, %1, %0" : "+v"(a) : "v"(b)))
DEF_OP(v_mul_f32, float, 1.0f + i * 1e-7f, asm volatile("v_mul_f32 %0, %1, %0" : "+v"(a) : "v"(b)))
DEF_OP(v_cvt_f32_u32, uint32_t, i, asm volatile("v_cvt_f32_u32 %0, %0" : "+v"(a)))
DEF_OP(v_fma_f32, float, 1.0f + i * 1e-7f, asm volatile("v_fma_f32 %0, %1, %1, %0" : "+v"(a) : "v"(b)))
DEF_OP(v_pk_fma_f32, f32x2, (f32x2{1.0f, 2.0f}), asm volatile("v_pk_fma_f32 %0, %1, %1, %0" : "+v"(a) : "v"(b)))
DEF_OP(v_fma_f64, double, 1.0 + i * 1e-9, asm volatile("v_fma_f64 %0, %1, %1, %0" : "+v"(a) : "v"(b)))
DEF_OP(v_mul_f64, double, 1.0 + i * 1e-9, asm volatile("v_mul_f64 %0, %1, %0" : "+v"(a) : "v"(b)))
DEF_OP(v_mul_lo_u32, uint32_t, i | 1u, asm volatile("v_mul_lo_u32 %0, %1, %0" : "+v"(a) : "v"(b)))
DEF_OP(v_mad_u64_u32, uint64_t, (uint64_t)i, { uint64_t c; asm volatile("v_mad_u64_u32 %0, %1, %2, %2, %0" : "+v"(a), "=s"(c) : "v"((uint32_t)b)); })
DEF_OP(v_bitop3_b32, uint32_t, i * 2654435761u, asm volatile("v_bitop3_b32 %0, %1, %0, %1 bitop3:0x96" : "+v"(a) : "v"(b)))
DEF_OP(v_cndmask_b32, uint32_t, i, asm volatile("v_cmp_gt_u32 vcc, %1, %0\n\tv_cndmask_b32 %0, %0, %1, vcc" : "+v"(a) : "v"(b) : "vcc"))
DEF_OP(v_rcp_f32, float, 1.0f + i * 1e-7f, asm volatile("v_rcp_f32 %0, %0" : "+v"(a)))
DEF_OP(v_exp_f32, float, i * 1e-9f, asm volatile("v_exp_f32 %0, %0" : "+v"(a)))
// round 3: the 4-wide node decode candidates (byte -> float conversions vs f16 mixes)
DEF_OP(v_cvt_f32_ubyte1, uint32_t, i, asm volatile("v_cvt_f32_ubyte1 %0, %0" : "+v"(a)))
DEF_OP(v_fma_mix_f32, float, 1.0f + i * 1e-7f, asm volatile("v_fma_mix_f32 %0, %1, %0, %0 op_sel_hi:[1,0,0]" : "+v"(a) : "v"(b)))
DEF_OP(v_perm_b32, uint32_t, i * 2654435761u, asm volatile("v_perm_b32 %0, %0, %1, %1" : "+v"(a) : "v"(b)))
DEF_OP(v_max3_f32, float, 1.0f + i * 1e-7f, asm volatile("v_max3_f32 %0, %1, %0, %1" : "+v"(a) : "v"(b)))
DEF_OP(v_min_f32, float, 1.0f + i * 1e-7f, asm volatile("v_min_f32 %0, %1, %0" : "+v"(a) : "v"(b)))
DEF_OP(v_pk_add_f32, f32x2, (f32x2{1.0f, 2.0f}), asm volatile("v_pk_add_f32 %0, %1, %0" : "+v"(a) : "v"(b)))
DEF_OP(v_pk_mul_f32, f32x2, (f32x2{1.0f, 2.0f}), asm volatile("v_pk_mul_f32 %0, %1, %0" : "+v"(a) : "v"(b)))
DEF_OP(v_fmac_f32, float, 1.0f + i * 1e-7f, asm volatile("v_fmac_f32 %0, %1, %1" : "+v"(a) : "v"(b)))
DEF_OP(v_cvt_f32_f16, uint32_t, i, asm volatile("v_cvt_f32_f16 %0, %0" : "+v"(a)))

template <class Op>
__global__ void __launch_bounds__(256) bench(uint64_t* out, uint32_t* sink) {
    using T = typename Op::type;
    T acc[CHAINS];
    const T b = Op::init(threadIdx.x + 7u);
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) acc[c] = Op::init(threadIdx.x * CHAINS + c);
    __syncthreads();
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    const uint64_t r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int u = 0; u < UNROLL; ++u)
#pragma unroll
            for (int c = 0; c < CHAINS; ++c) Op::step(acc[c], b);
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    const uint64_t r1 = __builtin_amdgcn_s_memrealtime();
    uint32_t h = 0;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) {
        uint32_t w = 0;
        __builtin_memcpy(&w, &acc[c], 4);
        h ^= w;
    }
    if (h == 0x12345678u) sink[0] = h;  // keep the chains live
    if ((threadIdx.x & 63u) == 0) {
        const uint32_t wv = blockIdx.x * 4 + threadIdx.x / 64;
        out[2 * wv] = t1 - t0;
        out[2 * wv + 1] = r1 - r0;
    }
}

template <class Op>
void run(int cus) {
    for (int W : {1, 4, 8}) {
        const int blocks = cus * W, waves = blocks * 4;
        uint64_t* d;
        uint32_t* s;
        hipMalloc(&d, waves * 2 * sizeof(uint64_t));
        hipMalloc(&s, 4);
        for (int rep = 0; rep < 3; ++rep) bench<Op><<<blocks, 256>>>(d, s);  // warm the clock
        hipEvent_t e0, e1;
        hipEventCreate(&e0);
        hipEventCreate(&e1);
        hipEventRecord(e0);
        bench<Op><<<blocks, 256>>>(d, s);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        std::vector<uint64_t> h(waves * 2);
        hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost);
        std::vector<double> cyc, clk;
        for (int k = 0; k < waves; ++k) {
            cyc.push_back((double)h[2 * k]);
            clk.push_back((double)h[2 * k] / (double)h[2 * k + 1] * 100.0);  // MHz
        }
        std::sort(cyc.begin(), cyc.end());
        std::sort(clk.begin(), clk.end());
        const double insts = (double)ITERS * UNROLL * CHAINS;
        const double med_cyc = cyc[cyc.size() / 2], med_clk = clk[clk.size() / 2];
        const double cpi = med_cyc / (W * insts);
        const double wall_rate = insts * waves / (ms * 1e-3) / (cus * 4.0);  // wave-insts / s / SIMD
        printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"cycles_per_wave_inst_per_simd\": %.3f, "
               "\"clock_mhz\": %.0f, \"wave_insts_per_s_per_simd\": %.4g, \"wall_wave_insts_per_s_per_simd\": %.4g, "
               "\"ms\": %.4f}\n",
               Op::name, W, cpi, med_clk, med_clk * 1e6 / cpi, wall_rate, ms);
        hipFree(d);
        hipFree(s);
    }
}

int main() {
    hipDeviceProp_t prop;
    hipGetDeviceProperties(&prop, 0);
    const int cus = prop.multiProcessorCount;
    printf("{\"device\": \"%s\", \"cus\": %d, \"clock_khz\": %d}\n", prop.gcnArchName, cus, prop.clockRate);
    run<v_xor_b32>(cus);
    run<v_add_f32>(cus);
    run<v_mul_f32>(cus);
    run<v_cvt_f32_u32>(cus);
    run<v_fma_f32>(cus);
    run<v_pk_fma_f32>(cus);
    run<v_fma_f64>(cus);
    run<v_mul_f64>(cus);
    run<v_mul_lo_u32>(cus);
    run<v_mad_u64_u32>(cus);
    run<v_bitop3_b32>(cus);
    run<v_cndmask_b32>(cus);
    run<v_rcp_f32>(cus);
    run<v_exp_f32>(cus);
    run<v_cvt_f32_ubyte1>(cus);
    run<v_fma_mix_f32>(cus);
    run<v_perm_b32>(cus);
    run<v_max3_f32>(cus);
    run<v_min_f32>(cus);
    run<v_pk_add_f32>(cus);
    run<v_pk_mul_f32>(cus);
    run<v_fmac_f32>(cus);
    run<v_cvt_f32_f16>(cus);
    return 0;
}
