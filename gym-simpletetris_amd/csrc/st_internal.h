// Internal declarations shared by the HIP kernels and the C-ABI layer.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "simpletetris.h"

namespace st {

constexpr int kWave = 64;      // one env per lane, one wave per workgroup
constexpr int kPad = 4;        // wall columns on each side of the LDS board
constexpr int kMaxW = 32;
constexpr int kMaxH = 28;
constexpr int kMtN = 624;
// Per-env MT storage (words): generation buffers A and B, then a 16-word pad
// (see st_kernels.hip, "Double-buffered twist"); 16-B aligned.
constexpr int64_t kMtPitch = 2 * kMtN + 16;
// after the last env: a draw window reads up to 16 words past index 623 of B
constexpr int64_t kMtPadBack = 64;
// diagnostic stamps per workgroup: st_step: logic wave 10 s_memtime phase
// stamps, s_memrealtime at start and end, HW_ID, XCC_ID, draw kind (words
// 0-15); draw wave 12 stamps + s_memrealtime at start and end (words 16-31);
// st_rollout: per-phase cycle totals of the logic / draw / output wave
// (words 0-15 / 16-31 / 32-47)
constexpr int kStampWords = 48;
constexpr int kPieceRow = ST_STAT_PIECE;     // rows 0..14 (counters + piece) move every step
constexpr int kHotRows = ST_STAT_PIECE + 1;
constexpr int kHotQ = (kHotRows * 16 + kWave - 1) / kWave;  // 16-B slots per lane

struct KParams {
    int32_t W, H;
    int32_t lock_mod;   // max(lock_delay, 0) + 1   (tetris_env.py:175)
    uint32_t flags;
    int32_t autoreset;
    uint32_t ablate;    // TIMING DIAGNOSTICS ONLY (env ST_ABLATE at st_create, read only by
                        // -DST_ABLATION=1 builds, tools/ablate.sh); 0 in
                        // every correct run: 1 = no lock path, 2 = no MT draw,
                        // 4 = no twist, 8 = no obs output; st_step: 1024 =
                        // counter rows read from the first workgroup's lines,
                        // 2048 = lock-path counter stores dropped, 4096 = board
                        // stores dropped, 8192 = late counter loads from the
                        // first workgroup's lines, 16384 / 32768 = the logic /
                        // draw wave's part of 2048 only; 65536 / 131072 = the
                        // draw wave's count / MT-word store only; 262144 = the draw
                        // wave's count rows T J L Z not loaded, 524288 = MT windows
                        // read as zeros, 1048576 = no next-generation chunks,
                        // 2097152 = the lock-path counter rows not loaded,
                        // 4194304 = the store phase's LDS transposition skipped
    uint64_t *stamps;   // DIAGNOSTIC build only (env ST_STAMPS at st_create): per-wave
                        // s_memtime at 8 phase boundaries of the step kernel
    int32_t k;          // st_rollout: number of steps
    int64_t n;          // real envs
    int64_t stride;     // padded env count (multiple of 64) = SoA row stride
    // state
    uint32_t *board;    // [W][stride]
    uint32_t *piece;    // [stride]
    int32_t *stats;     // [ST_NSTAT][stride]
    uint32_t *mt;       // [stride][kMtPitch]
    // io
    const uint8_t *actions;  // [n]
    const uint8_t *mask;     // [n] (reset) or null
    const uint64_t *seeds;   // [stride] (seed)
    uint32_t *obs;           // [W][n]
    float *obs_f32;          // [n][W][H]
    int32_t *reward;         // [n]
    uint8_t *done;           // [n]
    uint32_t *act_flag;      // st_set_action_flag: sticky "action outside 0..6" word, or null
    uint32_t *final_obs;     // st_step_vec: [W][n] terminal obs of envs reset in the step, or null
    uint32_t *wire;          // st_step_wire: [st_wire_words(W, H)][n] gather format, or null
    int32_t *info;           // st_step_vec: [ST_NSTAT][n] counters after the step, or null
    int32_t cus;             // compute units of the device (launch_rollout's kernel choice)
    // st_gate_actions: the step skips every env (no state change, no output)
    // when *gate == gate_epoch, i.e. the gate check before it saw an action
    // outside 0..6 (the reference's KeyError before any state change,
    // tetris_env.py:245); null: no gate (every launch but a gated one)
    const uint32_t *gate;
    uint32_t gate_epoch;
};

hipError_t launch_seed(const KParams &p, hipStream_t s);
hipError_t launch_reset(const KParams &p, hipStream_t s);
hipError_t launch_step(const KParams &p, hipStream_t s);
hipError_t launch_rollout(const KParams &p, hipStream_t s);
hipError_t launch_obs_f32(const KParams &p, const uint32_t *obs, float *out, hipStream_t s);
hipError_t launch_render(const KParams &p, hipStream_t s);
hipError_t launch_export(const KParams &p, int64_t env, const uint32_t *obs, const int32_t *rew,
                         const uint8_t *done, uint32_t parts, uint32_t *out, hipStream_t s);
hipError_t launch_mt_sync(const KParams &p, hipStream_t s);
hipError_t launch_policy_greedy(const KParams &p, uint64_t seed, int64_t t, uint32_t explore,
                                uint8_t *out, hipStream_t s);
hipError_t launch_grayscale(const KParams &p, const uint32_t *obs, int size, int channels,
                            int as_u8, void *out, hipStream_t s);
hipError_t launch_unwire(int W, int H, int64_t n_global, int shards, int64_t n_cap, const uint32_t *wire,
                         uint32_t *obs, int32_t *reward, uint8_t *done, hipStream_t s);
hipError_t launch_check_actions(const uint8_t *a, int64_t n, uint32_t *flag, hipStream_t s);
hipError_t launch_gate_actions(const uint8_t *a, int64_t n, uint32_t *words, uint32_t *host, uint32_t epoch,
                               hipStream_t s);
hipError_t launch_gen_actions(uint8_t *out, int64_t n, int64_t t, uint64_t seed, int64_t off,
                              hipStream_t s);

}  // namespace st
