// Multi-GPU render inside the library (SURVEY.md §8(b) "gpus", §8(e)): one process drives N
// devices; device r renders the image rows y = r (mod N) into HBM, then ONE RCCL gather
// (ncclGather over xGMI, rccl.h:745) brings the row shards to the first device, which
// un-permutes them into the frame.  The reference's Camera::render spreads one call over the
// whole machine (rayon's global pool, lib/camera.rs:315-316); this is that call for a node of
// MI355Xs.  nrt_render / nrt_render_device with nrt_render_opts.gpus = N reach it.
//
// Layout per context (one per (first device, N, loopback) of a scene), PIPE (4) buffer sets so frame
// k+1's renders can start while frame k's gather and un-permute run (and while frame k's slowest
// paths finish: the render streams of a device overlap one frame's tail with the next frame's
// start):
//   device d:  rows[PIPE]   (rows_max x W x 3 f32 each), render streams rs[STREAMS]; d >= 1 one comm
//              stream cs that carries every gather of its device in issue order (RCCL requires the
//              same order on every rank; one stream per communicator keeps it)
//   device 0:  staging[PIPE] (N x rows_max x W x 3 f32), the gather's receive buffers.  Its gathers
//              and the un-permute run on the CALLER's stream (nrt_render_device's hip_stream; the
//              context's host stream for nrt_render), chained to the previous frame's gather when
//              the caller switches streams, so device 0 runs the caller's stream + STREAMS (3)
//              render streams: a caller that copies the frame out on that same stream stays within
//              the process's 4 hardware queues (GPU_MAX_HW_QUEUES).
// One host thread enqueues all devices: every call here is asynchronous.
//
// N = 1 has nothing to exchange: its "gather" is a device-to-device copy into the staging buffer
// and no communicator is made.  (Measured on C5 through a communicator of one: ncclGather's kernel
// cost 0.12-0.3 ms of device time per 9.9-ms frame, 1.2-3 % -- more with fewer channels -- against
// 0.015 ms for the copy and the un-permute: the persistent render grid fills every CU, and the RCCL
// kernel's workgroups, 20 KB of LDS each, wait at the head of their queue for a render's tail.)
//
// Loopback (test only, NRT_MULTI_LOOPBACK=1 at context creation, api.cpp): the N logical shards all
// live on the first device, each with its own buffers and streams, and each shard's ncclGather is a
// device-to-device copy into the same staging slot on the same comm stream; everything else (row
// counts, short last shards, buffer-set rotation, event chaining, the un-permute) is the code the
// N-GPU render runs, so a one-GPU box exercises it.  bench.py refuses the mode.
//
// librccl is resolved with dlopen (soname librccl.so.1: the copy torch already loaded when it
// is in the process, else /opt/rocm's), so libnrt.so loads and renders on one device without it.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <unistd.h>  // types only: the functions come from dlopen below

#include <algorithm>
#include <cstdio>
#include <cstdlib>
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

// Render streams per device (frames rotate over them): 3, so device 0 runs the caller's stream + 3
// render streams = the process's 4 hardware queues when the caller copies the frame out on the same
// stream it passes (bench.py).  Buffer sets: one more than the streams.  The render kernel is
// persistent (its grid is the resident capacity), so the gather's kernel of frame k finds CU slots only
// when a later render's workgroups leave, at that render's tail; with sets = streams, frame k + 3's
// render waited for that gather, and a frame's tail went unfilled (C5 at N = 1 through RCCL: -1.2 %);
// with a spare set it waits for frame k - 1's gather, long done.  NRT_MULTI_STREAMS (1-3) and
// NRT_MULTI_PIPE (sets, >= streams, <= 4) at context creation for A/B runs.
constexpr int STREAMS = 3;
constexpr int PIPE = 4;  // (array capacity; sets in use default to the streams, NRT_MULTI_PIPE)
int env_int(const char* name, int dflt, int lo, int hi) {
    const char* e = std::getenv(name);
    const long v = e ? std::strtol(e, nullptr, 10) : dflt;
    return v >= lo && v <= hi ? (int)v : dflt;
}

// RCCL's first init prints a banner on stdout; the redirect around it swaps the process-wide fd 1,
// so two contexts created at once must not interleave it (one lock for every context)
std::mutex g_stdout_mu;

}  // namespace

struct MultiRender {
    int first = 0, n = 0;
    bool loopback = false;             // N logical shards on device `first` (test only)
    int pipe = PIPE;                   // buffer sets in use (<= PIPE)
    int nrs = STREAMS;                 // render streams per device in use (<= STREAMS, <= pipe)
    std::vector<DeviceScene*> scenes;  // scenes[d] lives on device dev_of(d)
    std::vector<ncclComm_t> comms;
    struct Dev {
        hipStream_t rs[STREAMS] = {};  // render streams (frames rotate)
        hipStream_t cs = nullptr;   // comm stream (every gather, in issue order); d = 0: the caller's
        float* rows[PIPE] = {};
        hipEvent_t rendered[PIPE] = {}, gathered[PIPE] = {};
        hipEvent_t t0[PIPE] = {}, t1[PIPE] = {};  // render kernel timing
    };
    std::vector<Dev> dev;
    float* staging[PIPE] = {};
    float* frame = nullptr;  // nrt_render's device frame on the first device
    hipStream_t host_stream = nullptr;  // device 0's comm stream for nrt_render (the host copy follows)
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
    int dev_of(int d) const { return loopback ? first : first + d; }
};

namespace {

void free_buffers(MultiRender* m) {
    for (int d = 0; d < m->n; ++d) {
        Guard g(m->dev_of(d));
        for (int s = 0; s < m->pipe; ++s) {
            if (m->dev[(size_t)d].rows[s]) (void)hipFree(m->dev[(size_t)d].rows[s]);
            m->dev[(size_t)d].rows[s] = nullptr;
        }
    }
    Guard g(m->first);
    for (int s = 0; s < m->pipe; ++s) {
        if (m->staging[s]) (void)hipFree(m->staging[s]);
        m->staging[s] = nullptr;
    }
    if (m->frame) (void)hipFree(m->frame);
    m->frame = nullptr;
    m->W = m->H = m->rows_max = 0;
}

// every enqueued frame done: the render and comm streams, and (device 0's gathers ran on callers'
// streams) the last gather event of every buffer set
void sync_all(MultiRender* m) {
    for (int d = 0; d < m->n; ++d) {
        Guard g(m->dev_of(d));
        const MultiRender::Dev& x = m->dev[(size_t)d];
        for (int s = 0; s < m->nrs; ++s)
            if (x.rs[s]) (void)hipStreamSynchronize(x.rs[s]);
        for (int s = 0; s < m->pipe; ++s)
            if (x.gathered[s]) (void)hipEventSynchronize(x.gathered[s]);
        if (x.cs) (void)hipStreamSynchronize(x.cs);
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
        Guard g(m->dev_of(d));
        for (int s = 0; s < m->pipe; ++s) {
            hcheck(hipMalloc((void**)&m->dev[(size_t)d].rows[s], shard), "hipMalloc(row shard)");
            hcheck(hipMemset(m->dev[(size_t)d].rows[s], 0, shard), "hipMemset(row shard)");  // rows past a short shard
        }
        hcheck(hipDeviceSynchronize(), "hipMemset(row shard)");  // (the render streams do not block on it)
    }
    Guard g(m->first);
    for (int s = 0; s < m->pipe; ++s) hcheck(hipMalloc((void**)&m->staging[s], shard * (size_t)m->n), "hipMalloc(staging)");
    m->W = W;
    m->H = H;
    m->rows_max = rows_max;
}

}  // namespace

MultiRender* gpu_multi_create(const std::vector<DeviceScene*>& scenes, bool loopback) {
    const Rccl& r = rccl();
    const bool need_rccl = !loopback && scenes.size() > 1;
    if (need_rccl && !r.ok) throw std::runtime_error("HIP error in multi-GPU render: " + r.why);
    if (scenes.empty()) throw std::invalid_argument("multi-GPU render: no devices");
    auto* m = new MultiRender();
    m->n = (int)scenes.size();
    m->loopback = loopback;
    m->nrs = env_int("NRT_MULTI_STREAMS", STREAMS, 1, STREAMS);
    m->pipe = env_int("NRT_MULTI_PIPE", m->nrs, m->nrs, PIPE);
    m->first = gpu_scene_device(scenes[0]);
    m->scenes = scenes;
    m->dev.resize(scenes.size());
    try {
        std::vector<int> devlist;
        for (int d = 0; d < m->n; ++d) {
            if (gpu_scene_device(scenes[(size_t)d]) != m->dev_of(d))
                throw std::invalid_argument(loopback ? "multi-GPU loopback: every shard renders on the first device"
                                                     : "multi-GPU render: devices must be consecutive ordinals");
            devlist.push_back(m->dev_of(d));
        }
        for (int d = 0; d < m->n; ++d) {
            Guard g(m->dev_of(d));
            MultiRender::Dev& x = m->dev[(size_t)d];
            for (int s = 0; s < m->nrs; ++s)
                hcheck(hipStreamCreateWithFlags(&x.rs[s], hipStreamNonBlocking), "hipStreamCreate");
            for (int s = 0; s < m->pipe; ++s) {
                hcheck(hipEventCreateWithFlags(&x.rendered[s], hipEventDisableTiming), "hipEventCreate");
                hcheck(hipEventCreateWithFlags(&x.gathered[s], hipEventDisableTiming), "hipEventCreate");
                hcheck(hipEventCreate(&x.t0[s]), "hipEventCreate");
                hcheck(hipEventCreate(&x.t1[s]), "hipEventCreate");
            }
            if (d > 0) hcheck(hipStreamCreateWithFlags(&x.cs, hipStreamNonBlocking), "hipStreamCreate");
        }
        {
            Guard g(m->first);
            hcheck(hipStreamCreateWithFlags(&m->host_stream, hipStreamNonBlocking), "hipStreamCreate");
            hcheck(hipEventCreate(&m->w0), "hipEventCreate");
            for (int s = 0; s < m->pipe; ++s) {
                hcheck(hipEventCreate(&m->g0[s]), "hipEventCreate");
                hcheck(hipEventCreate(&m->g1[s]), "hipEventCreate");
            }
        }
        if (need_rccl) {
            m->comms.assign((size_t)m->n, nullptr);
            // RCCL prints a version banner on stdout at its first init; a library keeps the caller's
            // stdout clean (bench.py's one JSON line, a CLI writing an image to stdout): the banner goes
            // to stderr
            std::lock_guard<std::mutex> lock(g_stdout_mu);
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
        }
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
        Guard g(m->dev_of(d));
        MultiRender::Dev& x = m->dev[(size_t)d];
        for (int s = 0; s < m->pipe; ++s) {
            for (hipEvent_t e : {x.rendered[s], x.gathered[s], x.t0[s], x.t1[s]})
                if (e) (void)hipEventDestroy(e);
        }
        for (int s = 0; s < m->nrs; ++s)
            if (x.rs[s]) (void)hipStreamDestroy(x.rs[s]);
        if (x.cs) (void)hipStreamDestroy(x.cs);
    }
    {
        Guard g(m->first);
        for (int s = 0; s < m->pipe; ++s)
            for (hipEvent_t e : {m->g0[s], m->g1[s]})
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
// device pointer on the first device) on `stream`, after its prior work.  `stream` is device 0's
// comm stream for this frame.
void enqueue(MultiRender* m, const RenderParams& p0, uint32_t precision, uint32_t rng, uint32_t trace, float* out,
             hipStream_t stream) {
    const Rccl& r = rccl();
    ensure_buffers(m, p0.width, p0.height);
    const int s = (int)(m->frames % (uint64_t)m->pipe);    // buffer set
    const int rsi = (int)(m->frames % (uint64_t)m->nrs);   // render stream
    const uint32_t N = (uint32_t)m->n;
    for (int d = 0; d < m->n; ++d) {
        Guard g(m->dev_of(d));
        MultiRender::Dev& x = m->dev[(size_t)d];
        hipStream_t rs = x.rs[rsi];
        // rows[s] is free once the gather of frame k - pipe has read it
        hcheck(hipStreamWaitEvent(rs, x.gathered[s], 0), "hipStreamWaitEvent");
        RenderParams q = p0;
        q.row_offset = (uint32_t)d;
        q.row_stride = N;
        q.rows = (uint32_t)d < p0.height ? (p0.height - (uint32_t)d + N - 1) / N : 0u;
        q.pixel_begin = 0;
        q.pixel_end = q.rows * q.width;
        q.out = x.rows[s];
        hcheck(hipEventRecord(x.t0[s], rs), "hipEventRecord");
        if (d == 0) {
            if (!m->w_armed) {
                hcheck(hipEventRecord(m->w0, rs), "hipEventRecord");
                m->w_armed = true;
                m->w_frames = 0;
            }
            ++m->w_frames;
        }
        if (q.rows) gpu_launch_render(m->scenes[(size_t)d], q, precision, rng, trace, rs);
        hcheck(hipEventRecord(x.t1[s], rs), "hipEventRecord");
        hcheck(hipEventRecord(x.rendered[s], rs), "hipEventRecord");
        hipStream_t cs = d == 0 ? stream : x.cs;
        hcheck(hipStreamWaitEvent(cs, x.rendered[s], 0), "hipStreamWaitEvent");
        // device 0's gathers run on the callers' streams: one that differs from the last frame's must
        // not start this gather before the previous one (RCCL's per-communicator order)
        if (d == 0 && m->last >= 0)
            hcheck(hipStreamWaitEvent(cs, x.gathered[m->last], 0), "hipStreamWaitEvent");
    }
    {
        Guard g(m->first);
        hcheck(hipEventRecord(m->g0[s], stream), "hipEventRecord");
    }
    const size_t count = (size_t)m->rows_max * m->W * 3;
    if (m->loopback || m->n == 1) {  // shard d's "gather": its rows into staging slot d, on its comm stream
        for (int d = 0; d < m->n; ++d) {
            Guard g(m->first);
            hcheck(hipMemcpyAsync(m->staging[s] + (size_t)d * count, m->dev[(size_t)d].rows[s], count * sizeof(float),
                                  hipMemcpyDeviceToDevice, d == 0 ? stream : m->dev[(size_t)d].cs),
                   "hipMemcpyAsync(loopback gather)");
        }
    } else {
        ncheck(r.group_start(), "ncclGroupStart");
        ncclResult_t gr = ncclSuccess;
        for (int d = 0; d < m->n && gr == ncclSuccess; ++d) {
            Guard g(m->dev_of(d));  // (RCCL's group launch reads the current device)
            gr = r.gather(m->dev[(size_t)d].rows[s], d == 0 ? m->staging[s] : nullptr, count, ncclFloat32, 0,
                          m->comms[(size_t)d], d == 0 ? stream : m->dev[(size_t)d].cs);
        }
        const ncclResult_t er = r.group_end();
        ncheck(gr, "ncclGather");
        ncheck(er, "ncclGroupEnd");
    }
    for (int d = 0; d < m->n; ++d) {
        Guard g(m->dev_of(d));
        hcheck(hipEventRecord(m->dev[(size_t)d].gathered[s], d == 0 ? stream : m->dev[(size_t)d].cs),
               "hipEventRecord");
    }
    Guard g(m->first);
    // RCCL's root completes its gather once every shard has arrived; the loopback copies of the other
    // shards ran on their own comm streams
    if (m->loopback)
        for (int d = 1; d < m->n; ++d)
            hcheck(hipStreamWaitEvent(stream, m->dev[(size_t)d].gathered[s], 0), "hipStreamWaitEvent");
    hipLaunchKernelGGL(unpermute_rows, dim3(m->H), dim3(256), 0, stream, (const float*)m->staging[s], out, N,
                       m->rows_max, m->W * 3u);
    hcheck(hipGetLastError(), "un-permute launch");
    hcheck(hipEventRecord(m->g1[s], stream), "hipEventRecord");
    m->last = s;
    ++m->frames;
}

// The caller's stream must belong to the first device (the null stream: the first device's).
void check_stream(const MultiRender* m, hipStream_t stream) {
    if (!stream) return;
    hipDevice_t d = -1;
    hcheck(hipStreamGetDevice(stream, &d), "hipStreamGetDevice");
    if ((int)d != m->first)
        throw std::invalid_argument("gpus >= 1: hip_stream belongs to device " + std::to_string((int)d) +
                                    ", the frame to device " + std::to_string(m->first) +
                                    " (opts.device; -1 = device 0)");
}

}  // namespace

void gpu_multi_render_device(MultiRender* m, const RenderParams& p, uint32_t precision, uint32_t rng, uint32_t trace,
                             float* dev_out, void* stream) {
    std::lock_guard<std::mutex> lock(m->mu);
    check_stream(m, (hipStream_t)stream);
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
            Guard g(m->dev_of(d));
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

void gpu_multi_prepare(MultiRender* m, uint32_t width, uint32_t height) {
    std::lock_guard<std::mutex> lock(m->mu);
    ensure_buffers(m, width, height);
}

bool gpu_multi_rccl_usable(std::string* why) {
    const Rccl& r = rccl();
    if (!r.ok && why) *why = r.why;
    return r.ok;
}

}  // namespace nrt
