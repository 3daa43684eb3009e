// Reference-exact kernels (Real = double).  Built with -ffp-contract=off so
// every f64 operation rounds exactly as the reference's Rust code does.
#include "kernel.hpp"
#include "launch.hpp"
#include "launch_impl.hpp"

namespace nrt {

void launch_exact(const RenderParams& p, const DSceneView<double>& v, uint32_t rng, int maxd, bool perlin,
                  bool planes, hipStream_t stream) {
    const bool deep = maxd > 1;
    if (rng == RNG_CHACHA8) {
        if (deep) launch_one<double, dev::ChaCha8, MAX_INSTANCE_DEPTH, true>(p, v, perlin, stream);
        else launch_one<double, dev::ChaCha8, 1, true>(p, v, perlin, stream, false, planes);
    } else {
        if (deep) launch_one<double, dev::Philox, MAX_INSTANCE_DEPTH, true>(p, v, perlin, stream);
        else launch_one<double, dev::Philox, 1, true>(p, v, perlin, stream);
    }
}

void launch_rng_probe(uint32_t rng, uint64_t stream0, uint32_t lanes, uint32_t count, uint32_t sample,
                      unsigned long long* d) {
    if (rng == RNG_CHACHA8)
        hipLaunchKernelGGL(dev::rng_probe_kernel<dev::ChaCha8>, dim3(1), dim3(lanes),
                           dev::RING * dev::BLOCK * sizeof(uint2), 0, stream0, count, sample, d);
    else if (rng == RNG_PHILOX)
        hipLaunchKernelGGL(dev::rng_probe_kernel<dev::Philox>, dim3(1), dim3(lanes), 0, 0, stream0, count, sample, d);
    else  // RNG_PHILOX2_BLOCK: the f32 render loop's blocks, word k = step k
        hipLaunchKernelGGL(dev::philox_block_probe_kernel<float>, dim3(1), dim3(lanes), 0, 0, (uint32_t)stream0, count,
                           sample, d);
}

}  // namespace nrt
