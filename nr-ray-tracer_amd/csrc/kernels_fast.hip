// Fast kernels (Real = float).  Built with -ffp-contract=fast; divisions on
// the hot path use the hardware reciprocal (kernel.hpp fast_div / fast_rcp).
#include "kernel.hpp"
#include "launch.hpp"
#include "launch_impl.hpp"

namespace nrt {

void launch_fast(const RenderParams& p, const DSceneView<float>& v, uint32_t rng, bool deep, hipStream_t stream) {
    if (rng == RNG_CHACHA8) {
        if (deep) launch_one<float, dev::ChaCha8, MAX_INSTANCE_DEPTH, false>(p, v, stream);
        else launch_one<float, dev::ChaCha8, 1, false>(p, v, stream);
    } else {
        if (deep) launch_one<float, dev::Philox, MAX_INSTANCE_DEPTH, false>(p, v, stream);
        else launch_one<float, dev::Philox, 1, false>(p, v, stream);
    }
}

}  // namespace nrt
