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

}  // namespace nrt
