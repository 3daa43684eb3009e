// Multi-GPU render inside the library (SURVEY.md §8(b) "gpus", §8(e)): one process drives N
// devices; device r renders the image rows y = r (mod N) into HBM, then ONE RCCL gather
// (ncclGather over xGMI, rccl.h:745) brings the row shards to the first device, which
// un-permutes them into the frame.  The reference's Camera::render spreads one call over the
// whole machine (rayon's global pool, lib/camera.rs:315-316); this is that call for a node of
// MI355Xs.  nrt_render / nrt_render_device with nrt_render_opts.gpus = N reach it.
//
// Layout per context (one per (first device, N) of a scene), PIPE buffer sets so frame k+1's
// renders can start while frame k's gather and un-permute run (and while frame k's slowest
// paths finish: the render streams of a device overlap one frame's tail with the next frame's
// start).  Two sets: three in flight measured N = 8 shards 0.931 -> 0.935-0.940 of linear but the
// whole C5 step 1-2 % slower (more streams than the process's 4 hardware queues: the host copy then
// shares a queue with a render):
//   device d:  rows[PIPE]   (rows_max x W x 3 f32 each), render streams rs[PIPE], one comm stream cs
//   device 0:  staging[PIPE] (N x rows_max x W x 3 f32), the gather's receive buffers
// The comm stream carries every gather of its device in issue order (RCCL requires the same
// order on every rank; one stream per communicator keeps it), after an event of the frame's
// render stream.  One host thread enqueues all devices: every call here is asynchronous.
//
// librccl is resolved with dlopen (soname librccl.so.1: the copy torch already loaded when it
// is in the process, else /opt/rocm's), so libnrt.so loads and renders on one device without it.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <unistd.h>  // types only: the functions come from dlopen below

#include <algorithm>
#include <cstdio>
#include <mutex>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <vector>

#include "gpu.hpp"
#include "nrt.h"

namespace nrt {
namespace {

void hcheck(hipError_t e, const char* what) {
    if (e != hipSuccess) throw std::runtime_error(std::string("HIP error in ") + what + ": " + hipGetErrorString(e));
}

struct Rccl {
    bool ok = false;
    std::string why;
    decltype(&ncclCommInitAll) init_all = nullptr;
    decltype(&ncclGather) gather = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclCommDestroy) destroy = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
};

const Rccl& rccl() {
    static const Rccl r = [] {
        Rccl x;
        void* h = nullptr;
        for (const char* name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"})
            if ((h = dlopen(name, RTLD_NOW | RTLD_LOCAL))) break;
        if (!h) {
            const char* e = dlerror();
            x.why = std::string("librccl not loadable: ") + (e ? e : "?");
            return x;
        }
        bool all = true;
        auto sym = [&](auto& fp, const char* name) {
            fp = reinterpret_cast<std::remove_reference_t<decltype(fp)>>(dlsym(h, name));
            all &= fp != nullptr;
        };
        sym(x.init_all, "ncclCommInitAll");
        sym(x.gather, "ncclGather");
        sym(x.group_start, "ncclGroupStart");
        sym(x.group_end, "ncclGroupEnd");
        sym(x.destroy, "ncclCommDestroy");
        sym(x.error_string, "ncclGetErrorString");
        x.ok = all;
        if (!all) x.why = "librccl lacks ncclGather / ncclCommInitAll (RCCL_GATHER_SCATTER)";
        return x;
    }();
    return r;
}

void ncheck(ncclResult_t r, const char* what) {
    if (r != ncclSuccess)
        throw std::runtime_error(std::string("HIP error in RCCL ") + what + ": " + rccl().error_string(r));
}

struct Guard {  // the caller's current device is restored (render.hip DeviceGuard)
    int prev = -1;
    explicit Guard(int d) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (d != prev) hcheck(hipSetDevice(d), "hipSetDevice");
    }
    ~Guard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

// Frame row y <- shard y % N, its row y / N.  One workgroup per frame row, 16-B moves when the
// row is a whole number of them (W x 3 floats: W % 4 == 0), else 4-B moves.
__global__ void __launch_bounds__(256) unpermute_rows(const float* __restrict__ staging, float* __restrict__ out,
                                                       uint32_t n_dev, uint32_t rows_max, uint32_t row_floats) {
    const uint32_t y = blockIdx.x;
    const float* src = staging + ((size_t)(y % n_dev) * rows_max + y / n_dev) * row_floats;
    float* dst = out + (size_t)y * row_floats;
    if ((row_floats & 3u) == 0) {
        const float4* s4 = reinterpret_cast<const float4*>(src);
        float4* d4 = reinterpret_cast<float4*>(dst);
        for (uint32_t i = threadIdx.x; i < row_floats / 4; i += blockDim.x) d4[i] = s4[i];
    } else {
        for (uint32_t i = threadIdx.x; i < row_floats; i += blockDim.x) dst[i] = src[i];
    }
}

constexpr int PIPE = 2;  // buffer sets (frames in flight)

}  // namespace

struct MultiRender {
    int first = 0, n = 0;
    std::vector<DeviceScene*> scenes;  // scenes[d] lives on device first + d
    std::vector<ncclComm_t> comms;
    struct Dev {
        hipStream_t rs[PIPE] = {};  // render streams (frames rotate)
        hipStream_t cs = nullptr;   // comm stream (every gather, in issue order)
        float* rows[PIPE] = {};
        hipEvent_t rendered[PIPE] = {}, gathered[PIPE] = {};
        hipEvent_t t0[PIPE] = {}, t1[PIPE] = {};  // render kernel timing
    };
    std::vector<Dev> dev;
    float* staging[PIPE] = {};
    float* frame = nullptr;  // nrt_render's device frame on the first device
    hipStream_t host_stream = nullptr;
    hipEvent_t in_ev[PIPE] = {}, done_ev[PIPE] = {};
    hipEvent_t g0[PIPE] = {}, g1[PIPE] = {};  // gather + un-permute timing
    // frame-period window (nrt_render_timings): w0 = the start of the first device's render of the
    // window's first frame, w_frames = frames enqueued in the window (consecutive frames' renders overlap,
    // so a window from a completion would miss the first frame's share and over-count the others)
    hipEvent_t w0 = nullptr;
    bool w_armed = false;
    uint64_t w_frames = 0;
    uint32_t W = 0, H = 0, rows_max = 0;
    uint64_t frames = 0;
    int last = -1;  // buffer set of the last frame
    std::mutex mu;
};

namespace {

void free_buffers(MultiRender* m) {
    for (int d = 0; d < m->n; ++d) {
        Guard g(m->first + d);
        for (int s = 0; s < PIPE; ++s) {
            if (m->dev[d].rows[s]) (void)hipFree(m->dev[d].rows[s]);
            m->dev[d].rows[s] = nullptr;
        }
    }
    Guard g(m->first);
    for (int s = 0; s < PIPE; ++s) {
        if (m->staging[s]) (void)hipFree(m->staging[s]);
        m->staging[s] = nullptr;
    }
    if (m->frame) (void)hipFree(m->frame);
    m->frame = nullptr;
    m->W = m->H = m->rows_max = 0;
}

void sync_all(MultiRender* m) {
    for (int d = 0; d < m->n; ++d) {
        Guard g(m->first + d);
        for (int s = 0; s < PIPE; ++s)
            if (m->dev[d].rs[s]) (void)hipStreamSynchronize(m->dev[d].rs[s]);
        if (m->dev[d].cs) (void)hipStreamSynchronize(m->dev[d].cs);
    }
    if (m->host_stream) {
        Guard g(m->first);
        (void)hipStreamSynchronize(m->host_stream);
    }
}

void ensure_buffers(MultiRender* m, uint32_t W, uint32_t H) {
    if (m->W == W && m->H == H) return;
    sync_all(m);
    free_buffers(m);
    const uint32_t rows_max = (H + (uint32_t)m->n - 1) / (uint32_t)m->n;
    const size_t shard = (size_t)rows_max * W * 3 * sizeof(float);
    for (int d = 0; d < m->n; ++d) {
        Guard g(m->first + d);
        for (int s = 0; s < PIPE; ++s) {
            hcheck(hipMalloc((void**)&m->dev[d].rows[s], shard), "hipMalloc(row shard)");
            hcheck(hipMemset(m->dev[d].rows[s], 0, shard), "hipMemset(row shard)");  // rows past a short shard
        }
    }
    Guard g(m->first);
    for (int s = 0; s < PIPE; ++s) hcheck(hipMalloc((void**)&m->staging[s], shard * (size_t)m->n), "hipMalloc(staging)");
    m->W = W;
    m->H = H;
    m->rows_max = rows_max;
}

}  // namespace

MultiRender* gpu_multi_create(const std::vector<DeviceScene*>& scenes) {
    const Rccl& r = rccl();
    if (!r.ok) throw std::runtime_error("HIP error in multi-GPU render: " + r.why);
    auto* m = new MultiRender();
    m->n = (int)scenes.size();
    m->first = gpu_scene_device(scenes[0]);
    m->scenes = scenes;
    m->dev.resize(scenes.size());
    try {
        std::vector<int> devlist;
        for (int d = 0; d < m->n; ++d) {
            if (gpu_scene_device(scenes[(size_t)d]) != m->first + d)
                throw std::invalid_argument("multi-GPU render: devices must be consecutive ordinals");
            devlist.push_back(m->first + d);
        }
        for (int d = 0; d < m->n; ++d) {
            Guard g(m->first + d);
            MultiRender::Dev& x = m->dev[(size_t)d];
            for (int s = 0; s < PIPE; ++s) {
                hcheck(hipStreamCreateWithFlags(&x.rs[s], hipStreamNonBlocking), "hipStreamCreate");
                hcheck(hipEventCreateWithFlags(&x.rendered[s], hipEventDisableTiming), "hipEventCreate");
                hcheck(hipEventCreateWithFlags(&x.gathered[s], hipEventDisableTiming), "hipEventCreate");
                hcheck(hipEventCreate(&x.t0[s]), "hipEventCreate");
                hcheck(hipEventCreate(&x.t1[s]), "hipEventCreate");
            }
            hcheck(hipStreamCreateWithFlags(&x.cs, hipStreamNonBlocking), "hipStreamCreate");
        }
        {
            Guard g(m->first);
            hcheck(hipStreamCreateWithFlags(&m->host_stream, hipStreamNonBlocking), "hipStreamCreate");
            hcheck(hipEventCreate(&m->w0), "hipEventCreate");
            for (int s = 0; s < PIPE; ++s) {
                hcheck(hipEventCreateWithFlags(&m->in_ev[s], hipEventDisableTiming), "hipEventCreate");
                hcheck(hipEventCreateWithFlags(&m->done_ev[s], hipEventDisableTiming), "hipEventCreate");
                hcheck(hipEventCreate(&m->g0[s]), "hipEventCreate");
                hcheck(hipEventCreate(&m->g1[s]), "hipEventCreate");
            }
        }
        m->comms.assign((size_t)m->n, nullptr);
        // RCCL prints a version banner on stdout at its first init; a library keeps the caller's
        // stdout clean (bench.py's one JSON line, a CLI writing an image to stdout): the banner goes
        // to stderr
        std::fflush(stdout);
        const int saved = ::dup(1);
        if (saved >= 0) (void)::dup2(2, 1);
        const ncclResult_t ir = r.init_all(m->comms.data(), m->n, devlist.data());
        std::fflush(stdout);
        if (saved >= 0) {
            (void)::dup2(saved, 1);
            ::close(saved);
        }
        ncheck(ir, "ncclCommInitAll");
    } catch (...) {
        gpu_multi_free(m);
        throw;
    }
    return m;
}

void gpu_multi_free(MultiRender* m) {
    if (!m) return;
    sync_all(m);
    for (ncclComm_t c : m->comms)
        if (c) (void)rccl().destroy(c);
    free_buffers(m);
    for (int d = 0; d < m->n; ++d) {
        Guard g(m->first + d);
        MultiRender::Dev& x = m->dev[(size_t)d];
        for (int s = 0; s < PIPE; ++s) {
            for (hipEvent_t e : {x.rendered[s], x.gathered[s], x.t0[s], x.t1[s]})
                if (e) (void)hipEventDestroy(e);
            if (x.rs[s]) (void)hipStreamDestroy(x.rs[s]);
        }
        if (x.cs) (void)hipStreamDestroy(x.cs);
    }
    {
        Guard g(m->first);
        for (int s = 0; s < PIPE; ++s)
            for (hipEvent_t e : {m->in_ev[s], m->done_ev[s], m->g0[s], m->g1[s]})
                if (e) (void)hipEventDestroy(e);
        if (m->w0) (void)hipEventDestroy(m->w0);
        if (m->host_stream) (void)hipStreamDestroy(m->host_stream);
    }
    delete m;
}

int gpu_multi_first(const MultiRender* m) { return m->first; }
int gpu_multi_count(const MultiRender* m) { return m->n; }

namespace {

// Enqueue one frame (caller holds m->mu): renders, the gather, the un-permute into `out` (a
// device pointer on the first device, ordered after `stream`'s prior work); `stream` waits for it.
void enqueue(MultiRender* m, const RenderParams& p0, uint32_t precision, uint32_t rng, uint32_t trace, float* out,
             hipStream_t stream) {
    const Rccl& r = rccl();
    ensure_buffers(m, p0.width, p0.height);
    const int s = (int)(m->frames % PIPE);
    const uint32_t N = (uint32_t)m->n;
    {
        Guard g(m->first);
        hcheck(hipEventRecord(m->in_ev[s], stream), "hipEventRecord");
    }
    for (int d = 0; d < m->n; ++d) {
        Guard g(m->first + d);
        MultiRender::Dev& x = m->dev[(size_t)d];
        // rows[s] is free once the gather of frame k - PIPE has read it
        hcheck(hipStreamWaitEvent(x.rs[s], x.gathered[s], 0), "hipStreamWaitEvent");
        RenderParams q = p0;
        q.row_offset = (uint32_t)d;
        q.row_stride = N;
        q.rows = (uint32_t)d < p0.height ? (p0.height - (uint32_t)d + N - 1) / N : 0u;
        q.pixel_begin = 0;
        q.pixel_end = q.rows * q.width;
        q.out = x.rows[s];
        hcheck(hipEventRecord(x.t0[s], x.rs[s]), "hipEventRecord");
        if (d == 0) {
            if (!m->w_armed) {
                hcheck(hipEventRecord(m->w0, x.rs[s]), "hipEventRecord");
                m->w_armed = true;
                m->w_frames = 0;
            }
            ++m->w_frames;
        }
        gpu_launch_render(m->scenes[(size_t)d], q, precision, rng, trace, x.rs[s]);
        hcheck(hipEventRecord(x.t1[s], x.rs[s]), "hipEventRecord");
        hcheck(hipEventRecord(x.rendered[s], x.rs[s]), "hipEventRecord");
        hcheck(hipStreamWaitEvent(x.cs, x.rendered[s], 0), "hipStreamWaitEvent");
    }
    {
        Guard g(m->first);
        hcheck(hipEventRecord(m->g0[s], m->dev[0].cs), "hipEventRecord");
    }
    const size_t count = (size_t)m->rows_max * m->W * 3;
    ncheck(r.group_start(), "ncclGroupStart");
    ncclResult_t gr = ncclSuccess;
    for (int d = 0; d < m->n && gr == ncclSuccess; ++d) {
        Guard g(m->first + d);  // (RCCL's group launch reads the current device)
        gr = r.gather(m->dev[(size_t)d].rows[s], d == 0 ? m->staging[s] : nullptr, count, ncclFloat32, 0,
                      m->comms[(size_t)d], m->dev[(size_t)d].cs);
    }
    const ncclResult_t er = r.group_end();
    ncheck(gr, "ncclGather");
    ncheck(er, "ncclGroupEnd");
    for (int d = 0; d < m->n; ++d) {
        Guard g(m->first + d);
        hcheck(hipEventRecord(m->dev[(size_t)d].gathered[s], m->dev[(size_t)d].cs), "hipEventRecord");
    }
    Guard g(m->first);
    hipStream_t cs0 = m->dev[0].cs;
    hcheck(hipStreamWaitEvent(cs0, m->in_ev[s], 0), "hipStreamWaitEvent");  // `out` is the caller's
    hipLaunchKernelGGL(unpermute_rows, dim3(m->H), dim3(256), 0, cs0, (const float*)m->staging[s], out, N,
                       m->rows_max, m->W * 3u);
    hcheck(hipGetLastError(), "un-permute launch");
    hcheck(hipEventRecord(m->g1[s], cs0), "hipEventRecord");
    hcheck(hipEventRecord(m->done_ev[s], cs0), "hipEventRecord");
    hcheck(hipStreamWaitEvent(stream, m->done_ev[s], 0), "hipStreamWaitEvent");
    m->last = s;
    ++m->frames;
}

}  // namespace

void gpu_multi_render_device(MultiRender* m, const RenderParams& p, uint32_t precision, uint32_t rng, uint32_t trace,
                             float* dev_out, void* stream) {
    std::lock_guard<std::mutex> lock(m->mu);
    enqueue(m, p, precision, rng, trace, dev_out, (hipStream_t)stream);
}

void gpu_multi_render_host(MultiRender* m, const RenderParams& p, uint32_t precision, uint32_t rng, uint32_t trace,
                           float* host_out) {
    std::lock_guard<std::mutex> lock(m->mu);
    ensure_buffers(m, p.width, p.height);
    const size_t bytes = (size_t)p.width * p.height * 3 * sizeof(float);
    Guard g(m->first);
    if (!m->frame) hcheck(hipMalloc((void**)&m->frame, bytes), "hipMalloc(frame)");
    enqueue(m, p, precision, rng, trace, m->frame, m->host_stream);
    hcheck(hipMemcpyAsync(host_out, m->frame, bytes, hipMemcpyDeviceToHost, m->host_stream), "hipMemcpyAsync(frame)");
    hcheck(hipStreamSynchronize(m->host_stream), "multi-GPU render");
}

size_t gpu_multi_timings(MultiRender* m, float* out, size_t n) {
    std::lock_guard<std::mutex> lock(m->mu);
    if (m->last < 0) throw std::invalid_argument("no multi-GPU render of this scene yet");
    const int s = m->last;
    for (int d = 0; d <= m->n + 1; ++d) {
        float ms = 0.0f;
        if (d < m->n) {
            Guard g(m->first + d);
            hcheck(hipEventSynchronize(m->dev[(size_t)d].t1[s]), "hipEventSynchronize");
            hcheck(hipEventElapsedTime(&ms, m->dev[(size_t)d].t0[s], m->dev[(size_t)d].t1[s]), "hipEventElapsedTime");
        } else if (d == m->n) {
            Guard g(m->first);
            hcheck(hipEventSynchronize(m->g1[s]), "hipEventSynchronize");
            hcheck(hipEventElapsedTime(&ms, m->g0[s], m->g1[s]), "hipEventElapsedTime");
        } else if (m->w_armed && m->w_frames > 1) {  // window start -> last completion, per frame
            Guard g(m->first);
            hcheck(hipEventElapsedTime(&ms, m->w0, m->g1[s]), "hipEventElapsedTime");
            ms /= (float)m->w_frames;
        }
        if ((size_t)d < n) out[d] = ms;
    }
    if (n > (size_t)m->n + 1) m->w_armed = false;  // read: the next frame opens a new window (a size query keeps it)
    return (size_t)m->n + 2;
}

}  // namespace nrt
