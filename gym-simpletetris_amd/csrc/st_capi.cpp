// st_capi.cpp -- extern "C" boundary of the batched SimpleTetris engine.
// Declared in include/simpletetris.h; each entry point cites the reference
// method it replaces there.  Owns the device state; launches the kernels of
// st_kernels.hip on the caller's stream.
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "st_internal.h"

struct st_ctx {
    st_config cfg;
    uint32_t ablate;
    uint64_t *stamps;
    int device;
    int64_t n;
    int64_t stride;
    bool seeded;
    bool reset_once;
    uint32_t *board;
    uint32_t *piece;
    int32_t *stats;
    uint32_t *mt;
    uint32_t *act_flag;  // st_set_action_flag (caller-owned), or null
    int cus;             // compute units of the device
    // st_gate_actions / st_gate_wait: the gate word (device), its host copy
    // (pinned, mapped), the event recorded behind the gate kernel, the last
    // epoch, and whether the next step launch is gated / a wait is pending
    uint32_t *gate;
    uint32_t *gate_host;
    uint32_t *gate_host_dev;
    hipEvent_t gate_ev;
    uint32_t gate_epoch;
    bool gate_armed;
    bool gate_pending;
};

namespace {

thread_local char g_err[512] = "";

int fail(int code, const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}

int hip_fail(hipError_t e, const char *what) {
    return fail(ST_EHIP, "%s: %s", what, hipGetErrorString(e));
}

#define ST_HIP(call)                                   \
    do {                                               \
        hipError_t _e = (call);                        \
        if (_e != hipSuccess) return hip_fail(_e, #call); \
    } while (0)

// Make the context's device current for the duration of a call.
struct DeviceGuard {
    int prev = -1;
    bool ok = true;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) ok = hipSetDevice(dev) == hipSuccess;
    }
    ~DeviceGuard() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

st::KParams params(const st_ctx *c) {
    st::KParams p{};
    p.W = c->cfg.width;
    p.H = c->cfg.height;
    p.lock_mod = (c->cfg.lock_delay > 0 ? c->cfg.lock_delay : 0) + 1;
    p.flags = c->cfg.flags;
    p.autoreset = c->cfg.autoreset;
    p.ablate = c->ablate;
    p.stamps = c->stamps;
    p.n = c->n;
    p.stride = c->stride;
    p.board = c->board;
    p.piece = c->piece;
    p.stats = c->stats;
    p.mt = c->mt;
    p.act_flag = c->act_flag;
    p.cus = c->cus;
    return p;
}

void free_state(st_ctx *c) {
    if (c->board) (void)hipFree(c->board);
    if (c->stats) (void)hipFree(c->stats);
    if (c->mt) (void)hipFree(c->mt);
    if (c->stamps) (void)hipFree(c->stamps);
    if (c->gate) (void)hipFree(c->gate);
    if (c->gate_host) (void)hipHostFree(c->gate_host);
    if (c->gate_ev) (void)hipEventDestroy(c->gate_ev);
    c->gate = c->gate_host = c->gate_host_dev = nullptr;
    c->gate_ev = nullptr;
    c->stamps = nullptr;
    c->board = c->piece = c->mt = nullptr;
    c->stats = nullptr;
}

}  // namespace

extern "C" {

const char *st_last_error(void) { return g_err; }
int st_abi_version(void) { return ST_ABI_VERSION; }

int st_create(st_ctx **out, const st_config *cfg, int device, int64_t n_envs) {
    g_err[0] = 0;
    if (!out || !cfg) return fail(ST_EINVAL, "st_create: null argument");
    *out = nullptr;
    if (cfg->width < 4 || cfg->width > st::kMaxW)
        return fail(ST_EINVAL, "width %d outside [4, %d]", cfg->width, st::kMaxW);
    if (cfg->height < 4 || cfg->height > st::kMaxH)
        return fail(ST_EINVAL, "height %d outside [4, %d]", cfg->height, st::kMaxH);
    if (cfg->lock_delay > 32766) return fail(ST_EINVAL, "lock_delay %d > 32766", cfg->lock_delay);
    if (cfg->flags & ~0xFFu) return fail(ST_EINVAL, "unknown flag bits 0x%x", cfg->flags);
    if (cfg->autoreset != ST_AUTORESET_NONE && cfg->autoreset != ST_AUTORESET_SAME_STEP)
        return fail(ST_EINVAL, "autoreset %d unknown", cfg->autoreset);
    if (n_envs < 1 || n_envs > (int64_t(1) << 24))  // 32-bit element offsets in the kernels
        return fail(ST_EINVAL, "n_envs %lld outside [1, 2^24] per context", (long long)n_envs);
    int ndev = 0;
    ST_HIP(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return fail(ST_EINVAL, "device %d of %d", device, ndev);
    DeviceGuard g(device);
    if (!g.ok) return fail(ST_EHIP, "hipSetDevice(%d) failed", device);

    st_ctx *c = new st_ctx();
    c->cfg = *cfg;
    c->device = device;
    if (const char *ab = getenv("ST_ABLATE")) c->ablate = (uint32_t)strtoul(ab, nullptr, 0);
    c->n = n_envs;
    if (hipDeviceGetAttribute(&c->cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) c->cus = 0;
    c->stride = (n_envs + st::kWave - 1) / st::kWave * st::kWave;
    const size_t sd = (size_t)c->stride;
    hipError_t e = hipSuccess;
    // board rows padded to a multiple of 4: a wave's 16-B accesses cover 4 rows
    const size_t wpad = (size_t)((cfg->width + 3) & ~3);
    if (e == hipSuccess) e = hipMalloc(&c->board, sd * wpad * sizeof(uint32_t));
    if (e == hipSuccess) e = hipMalloc(&c->stats, sd * ST_NSTAT * sizeof(int32_t));
    if (e == hipSuccess) c->piece = reinterpret_cast<uint32_t *>(c->stats) + ST_STAT_PIECE * sd;
    // MT states: [stride][kMtPitch] (+ the back pad a draw window may reach)
    if (e == hipSuccess) e = hipMalloc(&c->mt, (sd * st::kMtPitch + st::kMtPadBack) * sizeof(uint32_t));
    // diagnostic phase stamps (ST_STAMPS set: the instrumented step kernel)
    if (e == hipSuccess && getenv("ST_STAMPS"))
        e = hipMalloc(&c->stamps, (sd / st::kWave) * st::kStampWords * sizeof(uint64_t));
    if (e != hipSuccess) {
        free_state(c);
        delete c;
        return fail(ST_ENOMEM, "st_create: hipMalloc failed: %s", hipGetErrorString(e));
    }
    *out = c;
    return ST_OK;
}

int st_destroy(st_ctx *c) {
    if (!c) return ST_OK;
    DeviceGuard g(c->device);
    (void)hipDeviceSynchronize();
    free_state(c);
    delete c;
    return ST_OK;
}

int st_seed(st_ctx *c, const uint64_t *seeds_host, st_stream stream) {
    if (!c || !seeds_host) return fail(ST_EINVAL, "st_seed: null argument");
    DeviceGuard g(c->device);
    hipStream_t s = (hipStream_t)stream;
    // padding envs get seeds too (they run, unreported, in the last wave)
    uint64_t *d_seeds = nullptr;
    ST_HIP(hipMalloc(&d_seeds, (size_t)c->stride * sizeof(uint64_t)));
    hipError_t e = hipMemcpyAsync(d_seeds, seeds_host, (size_t)c->n * sizeof(uint64_t),
                                  hipMemcpyHostToDevice, s);
    if (e == hipSuccess && c->stride > c->n)
        e = hipMemsetAsync(d_seeds + c->n, 0, (size_t)(c->stride - c->n) * sizeof(uint64_t), s);
    st::KParams p = params(c);
    p.seeds = d_seeds;
    if (e == hipSuccess) e = st::launch_seed(p, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    (void)hipFree(d_seeds);
    if (e != hipSuccess) return hip_fail(e, "st_seed");
    c->seeded = true;
    return ST_OK;
}

int st_reset(st_ctx *c, const uint8_t *d_mask, st_stream stream) {
    if (!c) return fail(ST_EINVAL, "st_reset: null context");
    if (!c->seeded) return fail(ST_ESTATE, "st_reset before st_seed");
    DeviceGuard g(c->device);
    st::KParams p = params(c);
    p.mask = d_mask;
    ST_HIP(st::launch_reset(p, (hipStream_t)stream));
    if (!d_mask) c->reset_once = true;
    return ST_OK;
}

static int step_impl(st_ctx *c, const uint8_t *d_actions, uint32_t *d_obs, float *d_obs_f32,
                     int32_t *d_reward, uint8_t *d_done, st_stream stream, uint32_t *d_final_obs = nullptr,
                     int32_t *d_info = nullptr) {
    if (!c || !d_actions) return fail(ST_EINVAL, "st_step: null argument");
    if (!c->seeded || !c->reset_once)
        return fail(ST_ESTATE, "st_step before st_seed + st_reset (tetris_env.py:244 needs an anchor)");
    DeviceGuard g(c->device);
    st::KParams p = params(c);
    p.actions = d_actions;
    p.obs = d_obs;
    p.obs_f32 = d_obs_f32;
    p.reward = d_reward;
    p.done = d_done;
    p.final_obs = d_final_obs;
    p.info = d_info;
    if (c->gate_armed) {  // st_gate_actions ran for this step: skip it all if it saw a bad action
        p.gate = c->gate;
        p.gate_epoch = c->gate_epoch;
        c->gate_armed = false;
    }
    ST_HIP(st::launch_step(p, (hipStream_t)stream));
    return ST_OK;
}

int st_step(st_ctx *c, const uint8_t *d_actions, uint32_t *d_obs, int32_t *d_reward,
            uint8_t *d_done, st_stream stream) {
    return step_impl(c, d_actions, d_obs, nullptr, d_reward, d_done, stream);
}

int st_step_f32(st_ctx *c, const uint8_t *d_actions, uint32_t *d_obs, float *d_obs_f32,
                int32_t *d_reward, uint8_t *d_done, st_stream stream) {
    if (!d_obs_f32) return fail(ST_EINVAL, "st_step_f32: null d_obs_f32");
    return step_impl(c, d_actions, d_obs, d_obs_f32, d_reward, d_done, stream);
}

int st_step_n(st_ctx *c, const uint8_t *const *d_actions, int64_t k, uint32_t *d_obs, float *d_obs_f32,
              int32_t *d_reward, uint8_t *d_done, st_stream stream) {
    if (!c) return fail(ST_EINVAL, "st_step_n: null context");
    if (k <= 0) return ST_OK;
    if (!d_actions) return fail(ST_EINVAL, "st_step_n: null action pointer array");
    for (int64_t i = 0; i < k; ++i)
        if (!d_actions[i]) return fail(ST_EINVAL, "st_step_n: null action pointer");
    // one device switch for the whole loop (step_impl's own guard then finds
    // the device current and sets nothing)
    DeviceGuard g(c->device);
    for (int64_t i = 0; i < k; ++i) {
        const int rc = step_impl(c, d_actions[i], d_obs, d_obs_f32, d_reward, d_done, stream);
        if (rc != ST_OK) return rc;
    }
    return ST_OK;
}

int st_step_vec(st_ctx *c, const uint8_t *d_actions, uint32_t *d_obs, float *d_obs_f32, int32_t *d_reward,
                uint8_t *d_done, uint32_t *d_final_obs, int32_t *d_info, st_stream stream) {
    // final_obs is part of the obs output: without d_obs the kernel's two store
    // paths would disagree on whether it is written
    if (d_final_obs && !d_obs) return fail(ST_EINVAL, "st_step_vec: d_final_obs needs d_obs");
    return step_impl(c, d_actions, d_obs, d_obs_f32, d_reward, d_done, stream, d_final_obs, d_info);
}

int st_wire_words(int32_t width, int32_t height) {
    if (width < 1 || height < 1 || width > st::kMaxW || height > st::kMaxH)
        return fail(ST_EINVAL, "st_wire_words: board %dx%d outside 1..%d x 1..%d", width, height, st::kMaxW,
                    st::kMaxH);
    return (width * height + 33 + 31) / 32;
}

int st_step_wire(st_ctx *c, const uint8_t *d_actions, uint32_t *d_wire, st_stream stream) {
    if (!c || !d_actions || !d_wire) return fail(ST_EINVAL, "st_step_wire: null argument");
    if (!c->seeded || !c->reset_once)
        return fail(ST_ESTATE, "st_step_wire before st_seed + st_reset (tetris_env.py:244 needs an anchor)");
    DeviceGuard g(c->device);
    st::KParams p = params(c);
    p.actions = d_actions;
    p.wire = d_wire;
    ST_HIP(st::launch_step(p, (hipStream_t)stream));
    return ST_OK;
}

int st_unwire(int32_t width, int32_t height, int64_t n, const uint32_t *d_wire, uint32_t *d_obs,
              int32_t *d_reward, uint8_t *d_done, st_stream stream) {
    if (st_wire_words(width, height) < 0) return ST_EINVAL;
    if (n < 0) return fail(ST_EINVAL, "st_unwire: negative size");
    if (n > 0 && (!d_wire || !d_obs || !d_reward || !d_done)) return fail(ST_EINVAL, "st_unwire: null argument");
    ST_HIP(st::launch_unwire(width, height, n, 1, n, d_wire, d_obs, d_reward, d_done, (hipStream_t)stream));
    return ST_OK;
}

int st_unwire_shards(int32_t width, int32_t height, int64_t n_global, int32_t shards, int64_t n_cap,
                     const uint32_t *d_wire, uint32_t *d_obs, int32_t *d_reward, uint8_t *d_done, st_stream stream) {
    if (st_wire_words(width, height) < 0) return ST_EINVAL;
    if (n_global < 0 || shards < 1) return fail(ST_EINVAL, "st_unwire_shards: n_global < 0 or shards < 1");
    if (n_cap < (n_global + shards - 1) / shards)
        return fail(ST_EINVAL, "st_unwire_shards: n_cap %lld below the largest shard (%lld)", (long long)n_cap,
                    (long long)((n_global + shards - 1) / shards));
    if (n_global > 0 && (!d_wire || !d_obs || !d_reward || !d_done))
        return fail(ST_EINVAL, "st_unwire_shards: null argument");
    ST_HIP(st::launch_unwire(width, height, n_global, shards, n_cap, d_wire, d_obs, d_reward, d_done,
                             (hipStream_t)stream));
    return ST_OK;
}

int st_rollout(st_ctx *c, int32_t k, const uint8_t *d_actions, uint32_t *d_obs, float *d_obs_f32,
               int32_t *d_reward, uint8_t *d_done, st_stream stream) {
    if (!c || !d_actions) return fail(ST_EINVAL, "st_rollout: null argument");
    if (k < 1) return fail(ST_EINVAL, "st_rollout: k = %d < 1", k);
    if (!c->seeded || !c->reset_once)
        return fail(ST_ESTATE, "st_rollout before st_seed + st_reset (tetris_env.py:244 needs an anchor)");
    DeviceGuard g(c->device);
    st::KParams p = params(c);
    p.k = k;
    p.actions = d_actions;
    p.obs = d_obs;
    p.obs_f32 = d_obs_f32;
    p.reward = d_reward;
    p.done = d_done;
    ST_HIP(st::launch_rollout(p, (hipStream_t)stream));
    return ST_OK;
}

int st_mt_sync(st_ctx *c, st_stream stream) {
    if (!c) return fail(ST_EINVAL, "st_mt_sync: null context");
    DeviceGuard g(c->device);
    ST_HIP(st::launch_mt_sync(params(c), (hipStream_t)stream));
    return ST_OK;
}

int st_obs_to_f32(st_ctx *c, const uint32_t *d_obs, float *d_out, st_stream stream) {
    if (!c || !d_obs || !d_out) return fail(ST_EINVAL, "st_obs_to_f32: null argument");
    DeviceGuard g(c->device);
    ST_HIP(st::launch_obs_f32(params(c), d_obs, d_out, (hipStream_t)stream));
    return ST_OK;
}

int st_render(st_ctx *c, uint32_t *d_obs, st_stream stream) {
    if (!c || !d_obs) return fail(ST_EINVAL, "st_render: null argument");
    if (!c->seeded) return fail(ST_ESTATE, "st_render before st_seed");
    DeviceGuard g(c->device);
    st::KParams p = params(c);
    p.obs = d_obs;
    ST_HIP(st::launch_render(p, (hipStream_t)stream));
    return ST_OK;
}

int st_export_env(st_ctx *c, int64_t env, const uint32_t *d_obs, const int32_t *d_reward,
                  const uint8_t *d_done, uint32_t parts, uint32_t *d_out, st_stream stream) {
    if (!c || !d_out) return fail(ST_EINVAL, "st_export_env: null argument");
    if (env < 0 || env >= c->n) return fail(ST_EINVAL, "st_export_env: env %lld of %lld", (long long)env,
                                            (long long)c->n);
    if (parts & ~(ST_EXPORT_MT | ST_EXPORT_OBS_F32)) return fail(ST_EINVAL, "st_export_env: parts 0x%x", parts);
    if (!c->seeded) return fail(ST_ESTATE, "st_export_env before st_seed");
    DeviceGuard g(c->device);
    ST_HIP(st::launch_export(params(c), env, d_obs, d_reward, d_done, parts, d_out, (hipStream_t)stream));
    return ST_OK;
}

int st_export_words(int32_t width, int32_t height) {
    return width + 2 + ST_NSTAT + st::kMtN + width * height;
}

int st_grayscale(st_ctx *c, const uint32_t *d_obs, int32_t size, int32_t channels, int32_t as_u8,
                 void *d_out, st_stream stream) {
    if (!c || !d_obs || !d_out) return fail(ST_EINVAL, "st_grayscale: null argument");
    if (channels != 1 && channels != 3) return fail(ST_EINVAL, "channels %d not 1 or 3", channels);
    const int lim = c->cfg.width > c->cfg.height ? c->cfg.width : c->cfg.height;
    const int gap = size / 100 + 1;
    if (size < 8 || size > 4096 || (size - 2 * gap) / lim - gap < 1)
        return fail(ST_EINVAL, "st_grayscale: size %d too small for a %dx%d board", size,
                    c->cfg.width, c->cfg.height);
    DeviceGuard g(c->device);
    ST_HIP(st::launch_grayscale(params(c), d_obs, size, channels, as_u8, d_out, (hipStream_t)stream));
    return ST_OK;
}

int st_copy(void *dst, const void *src, int64_t bytes, st_stream stream) {
    if (bytes < 0 || ((!dst || !src) && bytes)) return fail(ST_EINVAL, "st_copy: bad argument");
    if (!bytes) return ST_OK;
    ST_HIP(hipMemcpyAsync(dst, src, (size_t)bytes, hipMemcpyDefault, (hipStream_t)stream));
    return ST_OK;
}

int st_state(st_ctx *c, st_state_views *out) {
    if (!c || !out) return fail(ST_EINVAL, "st_state: null argument");
    out->board = c->board;
    out->piece = c->piece;
    out->stats = c->stats;
    out->mt = c->mt;
    out->mt_pitch = st::kMtPitch;
    out->n_envs = c->n;
    out->stride = c->stride;
    out->width = c->cfg.width;
    out->height = c->cfg.height;
    return ST_OK;
}

namespace {
struct SnapHeader {  // st_save / st_load, 64 bytes
    char magic[8];
    uint32_t abi;  // the snapshot format version (kSnapVersion)
    int32_t width, height, nstat;
    int64_t n;
    uint8_t pad[32];
};
static_assert(sizeof(SnapHeader) == 64, "snapshot header");
const char kSnapMagic[8] = {'S', 'T', 'S', 'N', 'A', 'P', 0, 1};
// the snapshot format's own version (written where ABI 1 wrote its ABI
// version, 1): independent of ST_ABI_VERSION, which changes with the calls
constexpr uint32_t kSnapVersion = 1;

int64_t snap_bytes(const st_ctx *c) {
    return (int64_t)sizeof(SnapHeader) +
           c->n * 4 * ((int64_t)c->cfg.width + ST_NSTAT + st::kMtN);
}
}  // namespace

int64_t st_state_bytes(const st_ctx *c) { return c ? snap_bytes(c) : -1; }

int st_save(st_ctx *c, void *host_out, int64_t bytes) {
    if (!c || !host_out) return fail(ST_EINVAL, "st_save: null argument");
    if (bytes != snap_bytes(c))
        return fail(ST_EINVAL, "st_save: buffer is %lld bytes, a snapshot is %lld", (long long)bytes,
                    (long long)snap_bytes(c));
    DeviceGuard g(c->device);
    SnapHeader h{};
    memcpy(h.magic, kSnapMagic, sizeof(h.magic));
    h.abi = kSnapVersion;
    h.width = c->cfg.width;
    h.height = c->cfg.height;
    h.nstat = ST_NSTAT;
    h.n = c->n;
    char *o = static_cast<char *>(host_out);
    memcpy(o, &h, sizeof(h));
    o += sizeof(h);
    const size_t row = (size_t)c->n * 4, pitch = (size_t)c->stride * 4;
    ST_HIP(hipDeviceSynchronize());
    ST_HIP(st::launch_mt_sync(params(c), nullptr));  // CPython's MT state in the snapshot
    ST_HIP(hipDeviceSynchronize());
    ST_HIP(hipMemcpy2D(o, row, c->board, pitch, row, c->cfg.width, hipMemcpyDeviceToHost));
    o += row * c->cfg.width;
    ST_HIP(hipMemcpy2D(o, row, c->stats, pitch, row, ST_NSTAT, hipMemcpyDeviceToHost));
    o += row * ST_NSTAT;
    const size_t mrow = (size_t)st::kMtN * 4, mpitch = (size_t)st::kMtPitch * 4;
    ST_HIP(hipMemcpy2D(o, mrow, c->mt, mpitch, mrow, (size_t)c->n, hipMemcpyDeviceToHost));
    return ST_OK;
}

int st_load(st_ctx *c, const void *host_in, int64_t bytes) {
    if (!c || !host_in) return fail(ST_EINVAL, "st_load: null argument");
    if (bytes != snap_bytes(c))
        return fail(ST_EINVAL, "st_load: %lld bytes, this context's snapshot is %lld", (long long)bytes,
                    (long long)snap_bytes(c));
    SnapHeader h;
    memcpy(&h, host_in, sizeof(h));
    if (memcmp(h.magic, kSnapMagic, sizeof(h.magic)) != 0) return fail(ST_EINVAL, "st_load: not a snapshot");
    if (h.abi != kSnapVersion || h.nstat != ST_NSTAT)
        return fail(ST_EINVAL, "st_load: snapshot format %u (%d counter rows), this is %u (%d)", h.abi,
                    h.nstat, kSnapVersion, ST_NSTAT);
    if (h.width != c->cfg.width || h.height != c->cfg.height || h.n != c->n)
        return fail(ST_EINVAL, "st_load: snapshot of %lld %dx%d envs, context has %lld %dx%d",
                    (long long)h.n, h.width, h.height, (long long)c->n, c->cfg.width, c->cfg.height);
    const char *in = static_cast<const char *>(host_in) + sizeof(h);
    const size_t row = (size_t)c->n * 4, pitch = (size_t)c->stride * 4;
    {  // MT indexes must be CPython's (0..624): st_save writes them synced
        const int32_t *mi = reinterpret_cast<const int32_t *>(in + row * c->cfg.width) + ST_STAT_MT_INDEX * c->n;
        for (int64_t e = 0; e < c->n; ++e)
            if (mi[e] < 0 || mi[e] > st::kMtN)
                return fail(ST_EINVAL, "st_load: env %lld has MT index %d outside [0, 624]", (long long)e, mi[e]);
    }
    DeviceGuard g(c->device);
    ST_HIP(hipDeviceSynchronize());
    ST_HIP(hipMemcpy2D(c->board, pitch, in, row, row, c->cfg.width, hipMemcpyHostToDevice));
    in += row * c->cfg.width;
    ST_HIP(hipMemcpy2D(c->stats, pitch, in, row, row, ST_NSTAT, hipMemcpyHostToDevice));
    in += row * ST_NSTAT;
    const size_t mrow = (size_t)st::kMtN * 4, mpitch = (size_t)st::kMtPitch * 4;
    ST_HIP(hipMemcpy2D(c->mt, mpitch, in, mrow, mrow, (size_t)c->n, hipMemcpyHostToDevice));
    ST_HIP(hipDeviceSynchronize());
    c->seeded = c->reset_once = true;
    return ST_OK;
}

int st_debug_stamps(st_ctx *c, uint64_t *host_out, int64_t max_words) {
    if (!c || !host_out) return fail(ST_EINVAL, "st_debug_stamps: null argument");
    if (!c->stamps) return fail(ST_ESTATE, "context was not created with ST_STAMPS set");
    DeviceGuard g(c->device);
    int64_t n = (c->stride / st::kWave) * st::kStampWords;
    if (max_words < n) n = max_words;
    ST_HIP(hipDeviceSynchronize());
    ST_HIP(hipMemcpy(host_out, c->stamps, (size_t)n * sizeof(uint64_t), hipMemcpyDeviceToHost));
    return ST_OK;
}

int st_policy_greedy(st_ctx *c, uint64_t seed, int64_t t, uint32_t explore_permille, uint8_t *d_actions,
                     st_stream stream) {
    if (!c || !d_actions) return fail(ST_EINVAL, "st_policy_greedy: null argument");
    if (t < 0 || explore_permille > 1000) return fail(ST_EINVAL, "st_policy_greedy: t < 0 or explore > 1000");
    if (!c->seeded || !c->reset_once) return fail(ST_ESTATE, "st_policy_greedy before st_seed + st_reset");
    DeviceGuard g(c->device);
    ST_HIP(st::launch_policy_greedy(params(c), seed, t, explore_permille, d_actions, (hipStream_t)stream));
    return ST_OK;
}

int st_check_actions(const uint8_t *d_actions, int64_t n, uint32_t *d_flag, st_stream stream) {
    if (n < 0) return fail(ST_EINVAL, "st_check_actions: negative size");
    if (n > 0 && (!d_actions || !d_flag)) return fail(ST_EINVAL, "st_check_actions: null argument");
    ST_HIP(st::launch_check_actions(d_actions, n, d_flag, (hipStream_t)stream));
    return ST_OK;
}

int st_set_action_flag(st_ctx *c, uint32_t *d_flag) {
    if (!c) return fail(ST_EINVAL, "st_set_action_flag: null context");
    c->act_flag = d_flag;
    return ST_OK;
}

int st_gate_actions(st_ctx *c, const uint8_t *d_actions, st_stream stream) {
    if (!c || !d_actions) return fail(ST_EINVAL, "st_gate_actions: null argument");
    DeviceGuard g(c->device);
    if (!c->gate) {  // first use: the gate words (k_gate_actions), the mapped host word, the event
        ST_HIP(hipMalloc(&c->gate, 4 * sizeof(uint32_t)));
        ST_HIP(hipMemset(c->gate, 0, 4 * sizeof(uint32_t)));
        ST_HIP(hipHostMalloc(&c->gate_host, sizeof(uint32_t), hipHostMallocMapped | hipHostMallocCoherent));
        *c->gate_host = 0;
        void *dp = nullptr;
        ST_HIP(hipHostGetDevicePointer(&dp, c->gate_host, 0));
        c->gate_host_dev = static_cast<uint32_t *>(dp);
        ST_HIP(hipEventCreateWithFlags(&c->gate_ev, hipEventDisableTiming));
    }
    c->gate_epoch = (c->gate_epoch + 1u) & 0x7FFFFFFFu ? (c->gate_epoch + 1u) & 0x7FFFFFFFu : 1u;  // 31 bits, never 0
    hipStream_t s = (hipStream_t)stream;
    ST_HIP(st::launch_gate_actions(d_actions, c->n, c->gate, c->gate_host_dev, c->gate_epoch, s));  // gate = words[0]
    ST_HIP(hipEventRecord(c->gate_ev, s));
    c->gate_armed = true;
    c->gate_pending = true;
    return ST_OK;
}

int st_gate_wait(st_ctx *c) {
    if (!c) return fail(ST_EINVAL, "st_gate_wait: null context");
    if (!c->gate_pending) return fail(ST_ESTATE, "st_gate_wait without st_gate_actions");
    c->gate_pending = false;
    // the gate ends here: a step not launched by now (its launch failed, or
    // the caller never made it) is not gated by this check later
    c->gate_armed = false;
    // the gate kernel's last block writes epoch | bad << 31 to the mapped
    // host word (system scope): spin on it -- the wake-up of an event wait
    // costs more than the check itself -- and fall back to the event after
    // ~4 million polls (a few ms: the stream was busy with earlier work)
    const uint32_t ep = c->gate_epoch;
    for (int i = 0; i < (1 << 22); ++i) {
        const uint32_t v = __atomic_load_n(c->gate_host, __ATOMIC_ACQUIRE);
        if ((v & 0x7FFFFFFFu) == ep) return (int)(v >> 31);
        __builtin_ia32_pause();
    }
    DeviceGuard g(c->device);
    ST_HIP(hipEventSynchronize(c->gate_ev));
    const uint32_t v = __atomic_load_n(c->gate_host, __ATOMIC_ACQUIRE);
    if ((v & 0x7FFFFFFFu) != ep) return fail(ST_EHIP, "st_gate_wait: the gate kernel finished without its answer");
    return (int)(v >> 31);
}

int st_stream_wait(st_stream waiter, st_stream signaller) {
    if (waiter == signaller) return ST_OK;
    int dev = 0;
    ST_HIP(hipGetDevice(&dev));
    // one reusable event per (device, signalling stream) and thread: a wait
    // enqueued by hipStreamWaitEvent keeps the record it saw, so re-recording
    // the event for the next call is safe
    struct Ev {
        int dev;
        st_stream s;
        hipEvent_t ev;
    };
    thread_local Ev cache[16];
    thread_local int used = 0;
    hipEvent_t ev = nullptr;
    for (int i = 0; i < used; ++i)
        if (cache[i].dev == dev && cache[i].s == signaller) ev = cache[i].ev;
    if (!ev) {
        ST_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        if (used < 16) {
            cache[used++] = Ev{dev, signaller, ev};
        } else {  // evict the oldest entry
            (void)hipEventDestroy(cache[0].ev);
            for (int i = 1; i < 16; ++i) cache[i - 1] = cache[i];
            cache[15] = Ev{dev, signaller, ev};
        }
    }
    ST_HIP(hipEventRecord(ev, (hipStream_t)signaller));
    ST_HIP(hipStreamWaitEvent((hipStream_t)waiter, ev, 0));
    return ST_OK;
}

int st_stream_sync(st_stream stream) {
    ST_HIP(hipStreamSynchronize((hipStream_t)stream));
    return ST_OK;
}

int st_host_device_ptr(void *host, void **d_out) {
    if (!host || !d_out) return fail(ST_EINVAL, "st_host_device_ptr: null argument");
    *d_out = nullptr;
    ST_HIP(hipHostGetDevicePointer(d_out, host, 0));
    return ST_OK;
}

int st_gen_actions(uint8_t *d_out, int64_t n, int64_t t, uint64_t seed, int64_t global_offset,
                   st_stream stream) {
    if (!d_out && n > 0) return fail(ST_EINVAL, "st_gen_actions: null output");
    if (n < 0 || t < 0) return fail(ST_EINVAL, "st_gen_actions: negative size/time");
    ST_HIP(st::launch_gen_actions(d_out, n, t, seed, global_offset, (hipStream_t)stream));
    return ST_OK;
}

}  // extern "C"
