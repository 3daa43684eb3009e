// Fast kernels (Real = float).  Built with -ffp-contract=fast; divisions on
// the hot path use the hardware reciprocal (kernel.hpp fast_div / fast_rcp).
#include "kernel.hpp"
#include "launch.hpp"
#include "launch_impl.hpp"

namespace nrt {

template <class G>
static void launch_fast_rng(const RenderParams& p, const DSceneView<float>& v, int maxd, bool perlin, bool flat,
                            hipStream_t stream) {
    if (maxd == MODE_WORLD_BVH) launch_one<float, G, MODE_WORLD_BVH, false>(p, v, perlin, stream, flat);
    else if (maxd == MODE_WORLD_LIST) launch_one<float, G, MODE_WORLD_LIST, false>(p, v, perlin, stream, flat);
    else if (maxd == 1) launch_one<float, G, 1, false>(p, v, perlin, stream);
    else launch_one<float, G, MAX_INSTANCE_DEPTH, false>(p, v, perlin, stream);
}

void launch_fast(const RenderParams& p, const DSceneView<float>& v, uint32_t rng, int maxd, bool perlin, bool flat,
                 hipStream_t stream) {
    if (rng == RNG_CHACHA8) launch_fast_rng<dev::ChaCha8>(p, v, maxd, perlin, flat, stream);
    else launch_fast_rng<dev::Philox>(p, v, maxd, perlin, flat, stream);
}

void launch_fast_jit(const RenderParams& p0, const DSceneView<float>& v, void* fnp, uint32_t lds_fixed, int maxd,
                     uint32_t rng, uint32_t stack_entry, hipStream_t stream) {
    const hipFunction_t fn = (hipFunction_t)fnp;
    auto resident = [&](uint32_t lds) {
        return cached_resident((const void*)fn, lds, [&](int* per_cu) {
            return hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(per_cu, fn, dev::BLOCK, lds) == hipSuccess;
        });
    };
    auto launch = [&](uint32_t blocks, uint32_t lds, const RenderParams& p) {
        RenderParams pp = p;
        DSceneView<float> vv = v;
        void* args[] = {&pp, &vv};
        if (hipModuleLaunchKernel(fn, blocks, 1, 1, dev::BLOCK, 1, 1, lds, stream, args, nullptr) != hipSuccess)
            throw std::runtime_error("HIP error in hipModuleLaunchKernel (scene-specialised kernel)");
    };
    const uint32_t stack = maxd == MODE_WORLD_BVH ? (v.wbvh_stack + 1u) * dev::BLOCK * stack_entry : 0u;
    if (rng == RNG_CHACHA8) {  // persistent lanes (launch_variant): ring + stack below the staged scene
        const uint32_t npix = p0.pixel_end - p0.pixel_begin;
        uint32_t lds = lds_fixed + dev::chacha_lds_bytes(p0.exact_stage) + stack;
        RenderParams p = p0;
        exact_stage_fit(p, lds, resident);
        const uint64_t need = (npix + dev::BLOCK - 1) / dev::BLOCK;
        launch((uint32_t)std::max<uint64_t>(1, std::min<uint64_t>({need, resident(lds), chacha_grid_cap()})), lds, p);
        return;
    }
    if (maxd == MODE_WORLD_BVH)  // below the staged scene: the traversal stack (launch_one's ring)
        philox_launch<MODE_WORLD_BVH>(p0, lds_fixed + stack, resident, launch);
    else philox_launch<MODE_WORLD_LIST>(p0, lds_fixed, resident, launch);
}

}  // namespace nrt
