// bb_capi.cpp -- the C-ABI of include/bbvec.h on top of the gfx950 kernels.
//
// Owns the per-env device state (one hipMalloc slab, SoA columns aligned to
// 256 B), the piece tables and the numpy-exact seeding.  No compute happens on
// the host: there is no CPU fallback; every entry point that computes launches
// a HIP kernel and fails loudly when the device is unusable.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "bb_env_internal.h"

using namespace bb;

struct bb_env {
  int n = 0;
  int device = 0;
  int autoreset = 1;
  bb_reward_cfg cfg{};
  EnvDev d{};
  PieceRow* d_rows = nullptr;
  uint8_t* d_dtab = nullptr;
  JumpRow* d_jump = nullptr;
  void* slab = nullptr;
  int lane_budget = 16; // in-lane search budget before parking (BB_LANE_BUDGET; 0 = park every draw)
  int lane_quick = 2;   // in-lane test of 2 fixed slots (BB_LANE_QUICK; 0 = budget search instead)
  int pack_first = 8;   // escalate pass schedule (BB_PACK_FIRST / BB_PACK_NEXT, tuning only)
  int pack_next = 32;
  int dbg = 0;
  uint64_t* dbg_out = nullptr;
  // set when a bb_step launch failed: step_kernel may have parked envs (pend=1,
  // half-applied state) that escalate_kernel never finished; only a full
  // bb_reset (which clears every pend flag) makes the handle usable again
  bool broken = false;
  // bb_step through the rollout kernel (T = 1) instead of step + escalate kernels; the latter serves the
  // diagnostic modes (BB_DEBUG_MODE, BB_LANE_BUDGET, BB_LANE_QUICK) and BB_STEP_KERNELS=2
  bool fused_step = true;
  uint32_t* h_status = nullptr;  // device failure word (pinned, device-mapped): EnvDev::status, see kStatus*
  int64_t work_cap = 0;          // BB_DEBUG_ASYNC_CAP: rollout_async_kernel's working-iteration cap (tests only)
  std::string err;
};

static thread_local std::string g_create_err;

namespace {

int fail(bb_env* e, int code, const std::string& msg);

int broken_fail(bb_env* e, const char* what) {
  return fail(e, BB_ERR_STATE, std::string(what) + ": an earlier bb_step launch failed and left parked envs; "
                               "call bb_reset on all envs (d_env_mask = NULL) first");
}

int fail(bb_env* e, int code, const std::string& msg) {
  if (e) e->err = msg;
  else g_create_err = msg;
  return code;
}

int hip_fail(bb_env* e, hipError_t st, const char* what) {
  return fail(e, BB_ERR_HIP, std::string(what) + ": " + hipGetErrorString(st));
}

// A kernel raised the handle's status word (EnvDev::status): an earlier launch's outputs and the env state are
// incomplete.  The handle refuses work until a full bb_reset.  Reads the pinned word without synchronising, so
// it sees the launches that have finished by now (bb_sync waits for them first).
int status_fail(bb_env* e, const char* what) {
  const uint32_t st = __atomic_load_n(e->h_status, __ATOMIC_ACQUIRE);
  if (st == 0u) return BB_OK;
  e->broken = true;
  std::string why = st == kStatusAsyncCap
                        ? "a wave of rollout_async_kernel left through its iteration cap (a lost hand-search record): "
                          "that bb_rollout's outputs and the env state are incomplete"
                        : "device status " + std::to_string(st);
  return fail(e, BB_ERR_DEVICE, std::string(what) + ": " + why + "; call bb_reset on all envs (d_env_mask = NULL)");
}

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {}
};

template <typename T>
void carve(char*& cur, T*& out, size_t count) {
  out = reinterpret_cast<T*>(cur);
  size_t bytes = (count * sizeof(T) + 255) & ~size_t(255);
  cur += bytes;
}

size_t slab_bytes(int n) {
  size_t b = 0;
  auto add = [&](size_t count, size_t sz) { b += (count * sz + 255) & ~size_t(255); };
  add(n, 8);      // board
  add(n, 4);      // hand
  add(n, 8);      // score
  add(n, 4);      // combo
  add(n, 4);      // max_combo
  add(n, 4);      // moves
  add(n, 4);      // lines
  add(n, 4);      // blocks
  add(n, 2);      // prev
  add(3 * (size_t)n, 8);  // mask
  add(n, 8);      // rng_hi
  add(n, 8);      // rng_lo
  add(n, 4);      // rng_buf
  add(n, 8);      // inc_hi
  add(n, 8);      // inc_lo
  add(n, 8);      // seed_hi
  add(n, 8);      // seed_lo
  add(n, 1);      // has_seed
  add(n, 1);      // pend
  add(n, 8);      // pscratch
  add(kPieces, sizeof(PieceRow));
  add(kPieces * kPieces, 1);
  add(kJumpMax + 1, sizeof(JumpRow));
  return b;
}

// StepArgs fields that come from the handle (reward config, solver schedule).
StepArgs base_args(const bb_env* env) {
  StepArgs a{};
  a.cfg = env->cfg;
  a.center_tenth = env->cfg.center_bonus * 0.1;
  a.autoreset = env->autoreset;
  a.lane_budget = env->lane_budget;
  a.lane_quick = env->lane_quick;
  a.pack_first = env->pack_first;
  a.pack_next = env->pack_next;
  a.jump = env->d_jump;
  a.dbg = env->dbg;
  a.dbg_out = env->dbg_out;
  return a;
}

}  // namespace

// The build id (runtime/build.py: a hash of the sources, include/bbvec.h and the hipcc flags, passed as
// -DBB_BUILD_ID).  The marker prefix lets build.py read the id out of the .so without loading it.
#ifndef BB_BUILD_ID
#define BB_BUILD_ID "unhashed"
#endif
static const char kBuildIdMarker[] = "bbvec-build-id:" BB_BUILD_ID;

extern "C" {

int bb_abi_version(void) { return BB_ABI_VERSION; }

const char* bb_build_id(void) { return kBuildIdMarker + 15; }

const char* bb_last_error(const bb_env* env) { return env ? env->err.c_str() : g_create_err.c_str(); }

int32_t bb_num_envs(const bb_env* env) { return env ? env->n : 0; }

int bb_pcg64_seed(uint64_t seed, uint64_t out[4]) {
  if (!out) return BB_ERR_ARG;
  pcg64_seed_numpy(seed, out);
  return BB_OK;
}

int bb_create(int32_t num_envs, int32_t device, const bb_reward_cfg* cfg, int32_t autoreset, bb_env** out) {
  if (!out) return fail(nullptr, BB_ERR_ARG, "bb_create: out is NULL");
  *out = nullptr;
  if (num_envs <= 0) return fail(nullptr, BB_ERR_ARG, "bb_create: num_envs must be positive");
  if (!cfg) return fail(nullptr, BB_ERR_ARG, "bb_create: reward config is NULL");
  int ndev = 0;
  hipError_t st = hipGetDeviceCount(&ndev);
  if (st != hipSuccess || ndev <= 0)
    return fail(nullptr, BB_ERR_HIP, "bb_create: no HIP device available (this library has no CPU fallback)");
  if (device < 0 || device >= ndev) return fail(nullptr, BB_ERR_ARG, "bb_create: device index out of range");
  DeviceGuard g(device);
  bb_env* e = new bb_env();
  e->n = num_envs;
  e->device = device;
  e->autoreset = autoreset ? 1 : 0;
  e->cfg = *cfg;
  if (const char* s = getenv("BB_LANE_BUDGET")) e->lane_budget = atoi(s) > 0 ? atoi(s) : 0;
  if (const char* s = getenv("BB_DEBUG_MODE")) e->dbg = atoi(s);
  if (const char* s = getenv("BB_LANE_QUICK")) e->lane_quick = atoi(s) > 0 ? atoi(s) : 0;
  if (getenv("BB_LANE_BUDGET") && !getenv("BB_LANE_QUICK")) e->lane_quick = 0;  // explicit budget mode
  if (const char* s = getenv("BB_PACK_FIRST")) e->pack_first = atoi(s) > 0 ? atoi(s) : 1;
  if (const char* s = getenv("BB_PACK_NEXT")) e->pack_next = atoi(s) > 0 ? atoi(s) : 0;
  if (const char* s = getenv("BB_STEP_KERNELS")) e->fused_step = atoi(s) != 2;
  // the diagnostic modes and lane knobs exist only on the step + escalate kernels: they always win
  if (e->dbg || getenv("BB_LANE_BUDGET") || getenv("BB_LANE_QUICK")) e->fused_step = false;
  const size_t bytes = slab_bytes(num_envs);
  st = hipMalloc(&e->slab, bytes);
  if (st != hipSuccess) {
    std::string m = std::string("bb_create: hipMalloc: ") + hipGetErrorString(st);
    delete e;
    return fail(nullptr, BB_ERR_HIP, m);
  }
  (void)hipMemset(e->slab, 0, bytes);
  char* cur = static_cast<char*>(e->slab);
  const size_t n = (size_t)num_envs;
  EnvDev& d = e->d;
  d.n = num_envs;
  carve(cur, d.board, n);
  carve(cur, d.hand, n);
  carve(cur, d.score, n);
  carve(cur, d.combo, n);
  carve(cur, d.max_combo, n);
  carve(cur, d.moves, n);
  carve(cur, d.lines, n);
  carve(cur, d.blocks, n);
  carve(cur, d.prev, n);
  carve(cur, d.mask, 3 * n);
  carve(cur, d.rng_hi, n);
  carve(cur, d.rng_lo, n);
  carve(cur, d.rng_buf, n);
  carve(cur, d.inc_hi, n);
  carve(cur, d.inc_lo, n);
  carve(cur, d.seed_hi, n);
  carve(cur, d.seed_lo, n);
  carve(cur, d.has_seed, n);
  carve(cur, d.pend, n);
  carve(cur, d.pscratch, n);
  carve(cur, e->d_rows, kPieces);
  carve(cur, e->d_dtab, kPieces * kPieces);
  carve(cur, e->d_jump, kJumpMax + 1);
  PieceRow rows[kPieces];
  uint8_t dtab[kPieces * kPieces];
  JumpRow jump[kJumpMax + 1];
  build_piece_tables(rows, dtab);
  build_jump_table(jump);
  st = hipMemcpy(e->d_rows, rows, sizeof(rows), hipMemcpyHostToDevice);
  if (st == hipSuccess) st = hipMemcpy(e->d_dtab, dtab, sizeof(dtab), hipMemcpyHostToDevice);
  if (st == hipSuccess) st = hipMemcpy(e->d_jump, jump, sizeof(jump), hipMemcpyHostToDevice);
  if (st != hipSuccess) {
    std::string m = std::string("bb_create: table upload: ") + hipGetErrorString(st);
    (void)hipFree(e->slab);
    delete e;
    return fail(nullptr, BB_ERR_HIP, m);
  }
  if (const char* s = getenv("BB_DEBUG_ASYNC_CAP")) e->work_cap = atoll(s) > 0 ? atoll(s) : 0;
  st = hipHostMalloc(reinterpret_cast<void**>(&e->h_status), 64, hipHostMallocMapped | hipHostMallocCoherent);
  if (st == hipSuccess) {
    *e->h_status = 0u;
    st = hipHostGetDevicePointer(reinterpret_cast<void**>(&d.status), e->h_status, 0);
  }
  if (st != hipSuccess) {
    std::string m = std::string("bb_create: status word: ") + hipGetErrorString(st);
    if (e->h_status) (void)hipHostFree(e->h_status);
    (void)hipFree(e->slab);
    delete e;
    return fail(nullptr, BB_ERR_HIP, m);
  }
  if (e->dbg & 30) {
    if (hipMalloc(&e->dbg_out, n * 32) != hipSuccess) e->dbg &= ~30;
    else (void)hipMemset(e->dbg_out, 0, n * 32);
  }
  *out = e;
  return BB_OK;
}

void bb_destroy(bb_env* env) {
  if (!env) return;
  DeviceGuard g(env->device);
  if (env->slab) {
    (void)hipDeviceSynchronize();
    (void)hipFree(env->slab);
  }
  if (env->dbg_out) (void)hipFree(env->dbg_out);
  if (env->h_status) (void)hipHostFree(env->h_status);
  delete env;
}

int bb_seed(bb_env* env, const uint64_t* h_seeds, const uint8_t* h_has_seed, const uint64_t* h_raw) {
  if (!env) return BB_ERR_ARG;
  if (!h_has_seed) return fail(env, BB_ERR_ARG, "bb_seed: has_seed is NULL");
  const int n = env->n;
  std::vector<uint64_t> shi(n), slo(n), ihi(n), ilo(n);
  std::vector<uint8_t> has(n);
  for (int i = 0; i < n; ++i) {
    uint64_t w[4];
    if (h_has_seed[i] == 1) {
      if (!h_seeds) return fail(env, BB_ERR_ARG, "bb_seed: seeds is NULL");
      pcg64_seed_numpy(h_seeds[i], w);
    } else {
      if (!h_raw) return fail(env, BB_ERR_ARG, "bb_seed: raw state is NULL");
      for (int k = 0; k < 4; ++k) w[k] = h_raw[4 * (size_t)i + k];
      w[3] |= 1ull;  // PCG increments are odd
    }
    has[i] = h_has_seed[i] ? 1 : 0;
    shi[i] = w[0];
    slo[i] = w[1];
    ihi[i] = w[2];
    ilo[i] = w[3];
  }
  DeviceGuard g(env->device);
  hipError_t st = hipDeviceSynchronize();
  const size_t b8 = (size_t)n * 8;
  if (st == hipSuccess) st = hipMemcpy(env->d.seed_hi, shi.data(), b8, hipMemcpyHostToDevice);
  if (st == hipSuccess) st = hipMemcpy(env->d.seed_lo, slo.data(), b8, hipMemcpyHostToDevice);
  if (st == hipSuccess) st = hipMemcpy(env->d.rng_hi, shi.data(), b8, hipMemcpyHostToDevice);
  if (st == hipSuccess) st = hipMemcpy(env->d.rng_lo, slo.data(), b8, hipMemcpyHostToDevice);
  if (st == hipSuccess) st = hipMemcpy(env->d.inc_hi, ihi.data(), b8, hipMemcpyHostToDevice);
  if (st == hipSuccess) st = hipMemcpy(env->d.inc_lo, ilo.data(), b8, hipMemcpyHostToDevice);
  if (st == hipSuccess) st = hipMemcpy(env->d.has_seed, has.data(), (size_t)n, hipMemcpyHostToDevice);
  if (st == hipSuccess) st = hipMemset(env->d.rng_buf, 0, (size_t)n * 4);
  // clear has_uint32 in the hand words
  if (st == hipSuccess) st = hipMemset(env->d.hand, 0, (size_t)n * 4);
  if (st != hipSuccess) return hip_fail(env, st, "bb_seed");
  return BB_OK;
}

int bb_reset(bb_env* env, const uint8_t* d_env_mask, void* stream) {
  if (!env) return BB_ERR_ARG;
  if (env->broken && d_env_mask) return broken_fail(env, "bb_reset (masked)");
  if (d_env_mask && status_fail(env, "bb_reset (masked)") != BB_OK) return BB_ERR_DEVICE;
  DeviceGuard g(env->device);
  hipError_t st = hipSuccess;
  if (!d_env_mask) {
    // A full reset clears the status word in stream order: a rollout that is still queued or running ahead
    // of this reset may yet raise it, so the word is cleared only after that launch has finished -- by a
    // stream synchronisation and a host store, or (under graph capture, where a host sync is illegal) by a
    // device write queued on the stream.
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing((hipStream_t)stream, &cs) != hipSuccess) cs = hipStreamCaptureStatusNone;
    if (cs == hipStreamCaptureStatusNone) {
      st = hipStreamSynchronize((hipStream_t)stream);
      if (st == hipSuccess) __atomic_store_n(env->h_status, 0u, __ATOMIC_RELEASE);
    } else {
      st = hipMemsetAsync(env->d.status, 0, sizeof(uint32_t), (hipStream_t)stream);
    }
  }
  if (st == hipSuccess) st = launch_reset(env->d, env->d_rows, env->d_dtab, d_env_mask, (hipStream_t)stream);
  if (st != hipSuccess) return hip_fail(env, st, "bb_reset");
  if (!d_env_mask) env->broken = false;  // every env reset, every pend flag cleared
  return BB_OK;
}

int bb_step(bb_env* env, const int32_t* d_actions, const bb_step_out* out, void* stream) {
  if (!env) return BB_ERR_ARG;
  if (!d_actions || !out || !out->reward || !out->terminated)
    return fail(env, BB_ERR_ARG, "bb_step: actions, reward and terminated are required");
  StepArgs a = base_args(env);
  a.reward = out->reward;
  a.terminated = out->terminated;
  a.reward_f64 = out->reward_f64;
  a.mask_out = out->mask;
  a.lines = out->lines;
  a.info = out->info;
  a.next_action = out->next_action;
  a.policy_seed = out->policy_seed;
  a.policy_step = out->policy_step;
  a.env_offset = out->env_offset;
  a.final_score = out->final_score;
  a.final_moves = out->final_moves;
  DeviceGuard g(env->device);
  if (status_fail(env, "bb_step") != BB_OK) return BB_ERR_DEVICE;
  if (env->broken) return broken_fail(env, "bb_step");
  hipError_t st;
  if (env->fused_step) {
    // one launch: the rollout kernel at T = 1 (2 lanes per env, hand searches in the wave); output for
    // output equal to the two-kernel path below (tests/test_gpu_env_parity.py runs both)
    RollArgs r{};
    r.steps = 1;
    r.first_action = d_actions;
    r.reward = out->reward;
    r.terminated = out->terminated;
    r.lines = out->lines;
    r.mask = out->mask;
    r.next_action = out->next_action;
    r.policy_step0 = out->policy_step - 1;  // step 0's next action uses policy_step0 + 1
    r.info = out->info;
    r.reward_f64 = out->reward_f64;
    r.final_score = out->final_score;
    r.final_moves = out->final_moves;
    st = launch_rollout(env->d, env->d_rows, env->d_dtab, a, r, (hipStream_t)stream);
  } else {
    st = launch_step(env->d, env->d_rows, env->d_dtab, d_actions, a, (hipStream_t)stream);
  }
  if (st != hipSuccess) {
    env->broken = true;
    return hip_fail(env, st, "bb_step");
  }
  return BB_OK;
}

int bb_rollout(bb_env* env, int32_t steps, const int32_t* d_actions, const bb_rollout_out* out, void* stream) {
  if (!env) return BB_ERR_ARG;
  if (steps < 0) return fail(env, BB_ERR_ARG, "bb_rollout: steps must be >= 0");
  if (!d_actions || !out || !out->reward || !out->terminated)
    return fail(env, BB_ERR_ARG, "bb_rollout: actions, reward and terminated are required");
  if (env->dbg & ~16) return fail(env, BB_ERR_STATE, "bb_rollout: only BB_DEBUG_MODE=16 (rollout phase counters)");
  if (status_fail(env, "bb_rollout") != BB_OK) return BB_ERR_DEVICE;
  if (env->broken) return broken_fail(env, "bb_rollout");
  if (steps == 0) return BB_OK;
  StepArgs a = base_args(env);
  a.policy_seed = out->policy_seed;
  a.env_offset = out->env_offset;
  RollArgs r{};
  r.steps = steps;
  r.first_action = d_actions;
  r.reward = out->reward;
  r.terminated = out->terminated;
  r.lines = out->lines;
  r.actions = out->actions;
  r.mask = out->mask;
  r.next_action = out->next_action;
  r.policy_step0 = out->policy_step0;
  r.work_cap = env->work_cap;
  DeviceGuard g(env->device);
  hipError_t st = launch_rollout(env->d, env->d_rows, env->d_dtab, a, r, (hipStream_t)stream);
  if (st != hipSuccess) return hip_fail(env, st, "bb_rollout");
  return BB_OK;
}

int bb_sync(bb_env* env, void* stream) {
  if (!env) return BB_ERR_ARG;
  DeviceGuard g(env->device);
  const hipError_t st = hipStreamSynchronize((hipStream_t)stream);
  if (st != hipSuccess) return hip_fail(env, st, "bb_sync");
  return status_fail(env, "bb_sync");
}

int bb_obs(bb_env* env, float* d_x, int8_t* d_mask_i8, float* d_mask_f32, uint64_t* d_mask_bits, void* stream) {
  if (!env) return BB_ERR_ARG;
  if (status_fail(env, "bb_obs") != BB_OK) return BB_ERR_DEVICE;  // the state an incomplete launch left
  if (env->broken) return broken_fail(env, "bb_obs");
  DeviceGuard g(env->device);
  hipStream_t s = (hipStream_t)stream;
  hipError_t st = launch_expand(env->d.board, env->d.hand, env->d.mask, nullptr, env->d_rows, env->n, d_x,
                                d_mask_f32, d_mask_i8, s);
  if (st == hipSuccess && d_mask_bits)
    st = hipMemcpyAsync(d_mask_bits, env->d.mask, (size_t)env->n * 24, hipMemcpyDeviceToDevice, s);
  if (st != hipSuccess) return hip_fail(env, st, "bb_obs");
  return BB_OK;
}

int bb_device_ptrs(bb_env* env, uint64_t** d_board, uint32_t** d_hand, uint64_t** d_mask) {
  if (!env) return BB_ERR_ARG;
  if (d_board) *d_board = env->d.board;
  if (d_hand) *d_hand = env->d.hand;
  if (d_mask) *d_mask = env->d.mask;
  return BB_OK;
}

int bb_snapshot(bb_env* env, uint64_t* d_board, uint32_t* d_hand, uint64_t* d_mask_bits, void* stream) {
  if (!env) return BB_ERR_ARG;
  if (status_fail(env, "bb_snapshot") != BB_OK) return BB_ERR_DEVICE;
  if (env->broken) return broken_fail(env, "bb_snapshot");
  DeviceGuard g(env->device);
  hipStream_t s = (hipStream_t)stream;
  const size_t n = (size_t)env->n;
  hipError_t st = hipSuccess;
  if (d_board) st = hipMemcpyAsync(d_board, env->d.board, n * 8, hipMemcpyDeviceToDevice, s);
  if (st == hipSuccess && d_hand) st = hipMemcpyAsync(d_hand, env->d.hand, n * 4, hipMemcpyDeviceToDevice, s);
  if (st == hipSuccess && d_mask_bits)
    st = hipMemcpyAsync(d_mask_bits, env->d.mask, n * 24, hipMemcpyDeviceToDevice, s);
  if (st != hipSuccess) return hip_fail(env, st, "bb_snapshot");
  return BB_OK;
}

int bb_get_state(bb_env* env, const bb_state_view* v) {
  if (!env || !v) return BB_ERR_ARG;
  DeviceGuard g(env->device);
  const size_t n = (size_t)env->n;
  hipError_t st = hipDeviceSynchronize();
  auto cp = [&](void* dst, const void* src, size_t bytes) {
    if (dst && st == hipSuccess) st = hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost);
  };
  if (st == hipSuccess && status_fail(env, "bb_get_state") != BB_OK) return BB_ERR_DEVICE;
  cp(v->board, env->d.board, n * 8);
  cp(v->hand, env->d.hand, n * 4);
  cp(v->score, env->d.score, n * 8);
  cp(v->combo, env->d.combo, n * 4);
  cp(v->max_combo, env->d.max_combo, n * 4);
  cp(v->moves, env->d.moves, n * 4);
  cp(v->lines, env->d.lines, n * 4);
  cp(v->blocks, env->d.blocks, n * 4);
  if ((v->prev_holes || v->prev_center) && st == hipSuccess) {
    std::vector<uint16_t> prev(n);
    st = hipMemcpy(prev.data(), env->d.prev, n * 2, hipMemcpyDeviceToHost);
    for (size_t i = 0; i < n && st == hipSuccess; ++i) {
      if (v->prev_holes) v->prev_holes[i] = (uint8_t)(prev[i] & 0xFF);
      if (v->prev_center) v->prev_center[i] = (uint8_t)(prev[i] >> 8);
    }
  }
  if (v->rng && st == hipSuccess) {
    std::vector<uint64_t> hi(n), lo(n);
    std::vector<uint32_t> buf(n);
    st = hipMemcpy(hi.data(), env->d.rng_hi, n * 8, hipMemcpyDeviceToHost);
    if (st == hipSuccess) st = hipMemcpy(lo.data(), env->d.rng_lo, n * 8, hipMemcpyDeviceToHost);
    if (st == hipSuccess) st = hipMemcpy(buf.data(), env->d.rng_buf, n * 4, hipMemcpyDeviceToHost);
    for (size_t i = 0; i < n && st == hipSuccess; ++i) {
      v->rng[3 * i] = hi[i];
      v->rng[3 * i + 1] = lo[i];
      v->rng[3 * i + 2] = buf[i];
    }
  }
  if (st != hipSuccess) return hip_fail(env, st, "bb_get_state");
  return BB_OK;
}

int bb_set_state(bb_env* env, const bb_state_view* v) {
  if (!env || !v) return BB_ERR_ARG;
  DeviceGuard g(env->device);
  const size_t n = (size_t)env->n;
  hipError_t st = hipDeviceSynchronize();
  auto cp = [&](void* dst, const void* src, size_t bytes) {
    if (src && st == hipSuccess) st = hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice);
  };
  cp(env->d.board, v->board, n * 8);
  cp(env->d.hand, v->hand, n * 4);
  cp(env->d.score, v->score, n * 8);
  cp(env->d.combo, v->combo, n * 4);
  cp(env->d.max_combo, v->max_combo, n * 4);
  cp(env->d.moves, v->moves, n * 4);
  cp(env->d.lines, v->lines, n * 4);
  cp(env->d.blocks, v->blocks, n * 4);
  if ((v->prev_holes || v->prev_center) && st == hipSuccess) {
    std::vector<uint16_t> prev(n);
    st = hipMemcpy(prev.data(), env->d.prev, n * 2, hipMemcpyDeviceToHost);
    for (size_t i = 0; i < n; ++i) {
      uint16_t h = v->prev_holes ? v->prev_holes[i] : (uint16_t)(prev[i] & 0xFF);
      uint16_t c = v->prev_center ? v->prev_center[i] : (uint16_t)(prev[i] >> 8);
      prev[i] = (uint16_t)(h | (c << 8));
    }
    if (st == hipSuccess) st = hipMemcpy(env->d.prev, prev.data(), n * 2, hipMemcpyHostToDevice);
  }
  if (v->rng && st == hipSuccess) {
    std::vector<uint64_t> hi(n), lo(n);
    std::vector<uint32_t> buf(n);
    for (size_t i = 0; i < n; ++i) {
      hi[i] = v->rng[3 * i];
      lo[i] = v->rng[3 * i + 1];
      buf[i] = (uint32_t)v->rng[3 * i + 2];
    }
    st = hipMemcpy(env->d.rng_hi, hi.data(), n * 8, hipMemcpyHostToDevice);
    if (st == hipSuccess) st = hipMemcpy(env->d.rng_lo, lo.data(), n * 8, hipMemcpyHostToDevice);
    if (st == hipSuccess) st = hipMemcpy(env->d.rng_buf, buf.data(), n * 4, hipMemcpyHostToDevice);
  }
  // the mask column is derived state: recompute it from board + hand
  if (st == hipSuccess && (v->board || v->hand)) {
    st = launch_refresh_mask(env->d, env->d_rows, nullptr);
    if (st == hipSuccess) st = hipDeviceSynchronize();
  }
  if (st != hipSuccess) return hip_fail(env, st, "bb_set_state");
  return BB_OK;
}

int bb_debug_counters(bb_env* env, uint64_t* h_out) {
  if (!env || !h_out) return BB_ERR_ARG;
  if (!env->dbg_out) return fail(env, BB_ERR_STATE, "bb_debug_counters: create with BB_DEBUG_MODE bit 1 or 2 set");
  DeviceGuard g(env->device);
  hipError_t st = hipDeviceSynchronize();
  if (st == hipSuccess) st = hipMemcpy(h_out, env->dbg_out, (size_t)env->n * 32, hipMemcpyDeviceToHost);
  if (st == hipSuccess) st = hipMemset(env->dbg_out, 0, (size_t)env->n * 32);
  if (st != hipSuccess) return hip_fail(env, st, "bb_debug_counters");
  return BB_OK;
}

int bb_random_actions(const uint64_t* d_mask_bits, int32_t n, uint64_t seed, uint64_t step, uint64_t env_offset,
                      int32_t* d_actions, void* stream) {
  if (!d_mask_bits || !d_actions || n < 0) return fail(nullptr, BB_ERR_ARG, "bb_random_actions: bad arguments");
  hipError_t st = launch_random_actions(d_mask_bits, n, seed, step, env_offset, d_actions, (hipStream_t)stream);
  if (st != hipSuccess) return fail(nullptr, BB_ERR_HIP, std::string("bb_random_actions: ") + hipGetErrorString(st));
  return BB_OK;
}

int bb_masked_sample(const float* d_logits, const uint64_t* d_mask_bits, int32_t n, const float* d_uniform,
                     uint64_t seed, uint64_t step, uint64_t env_offset, int32_t deterministic,
                     const int64_t* d_action_in, int64_t* d_action, float* d_logp, float* d_entropy,
                     void* stream) {
  if (!d_logits || !d_mask_bits || n < 0) return fail(nullptr, BB_ERR_ARG, "bb_masked_sample: bad arguments");
  if (n == 0) return BB_OK;
  hipError_t st = launch_masked_sample(d_logits, d_mask_bits, n, d_uniform, seed, step, nullptr, env_offset, deterministic,
                                       d_action_in, d_action, d_logp, d_entropy, (hipStream_t)stream);
  if (st != hipSuccess) return fail(nullptr, BB_ERR_HIP, std::string("bb_masked_sample: ") + hipGetErrorString(st));
  return BB_OK;
}

int bb_masked_sample_dstep(const float* d_logits, const uint64_t* d_mask_bits, int32_t n, uint64_t seed,
                           const uint64_t* d_step, uint64_t step_add, uint64_t env_offset, int32_t deterministic,
                           int64_t* d_action, float* d_logp, float* d_entropy, void* stream) {
  if (!d_logits || !d_mask_bits || !d_step || n < 0)
    return fail(nullptr, BB_ERR_ARG, "bb_masked_sample_dstep: bad arguments");
  if (n == 0) return BB_OK;
  hipError_t st = launch_masked_sample(d_logits, d_mask_bits, n, nullptr, seed, step_add, d_step, env_offset,
                                       deterministic, nullptr, d_action, d_logp, d_entropy, (hipStream_t)stream);
  if (st != hipSuccess)
    return fail(nullptr, BB_ERR_HIP, std::string("bb_masked_sample_dstep: ") + hipGetErrorString(st));
  return BB_OK;
}

int bb_gae(const float* d_rewards, const float* d_values, const float* d_dones, const float* d_last_values, int32_t T,
           int32_t N, float gamma, float gamma_lambda, float* d_adv, float* d_ret, void* stream) {
  if (!d_rewards || !d_values || !d_dones || !d_last_values || !d_adv || !d_ret || T <= 0 || N <= 0)
    return fail(nullptr, BB_ERR_ARG, "bb_gae: bad arguments");
  hipError_t st = launch_gae(d_rewards, d_values, d_dones, d_last_values, T, N, gamma, gamma_lambda, d_adv, d_ret,
                             (hipStream_t)stream);
  if (st != hipSuccess) return fail(nullptr, BB_ERR_HIP, std::string("bb_gae: ") + hipGetErrorString(st));
  return BB_OK;
}

int bb_gather_obs(const uint64_t* d_board, const uint32_t* d_hand, const uint64_t* d_mask_bits,
                  const int64_t* d_index, int32_t n, float* d_x, float* d_mask_f32, void* stream) {
  if (n < 0 || (d_x && (!d_board || !d_hand)) || (d_mask_f32 && !d_mask_bits))
    return fail(nullptr, BB_ERR_ARG, "bb_gather_obs: bad arguments");
  if (n == 0) return BB_OK;
  static PieceRow* s_rows = nullptr;  // per-process copy of the table for the stateless gather
  static int s_dev = -1;
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (!s_rows || s_dev != dev) {
    PieceRow rows[kPieces];
    uint8_t dtab[kPieces * kPieces];
    build_piece_tables(rows, dtab);
    hipError_t st = hipMalloc(&s_rows, sizeof(rows));
    if (st == hipSuccess) st = hipMemcpy(s_rows, rows, sizeof(rows), hipMemcpyHostToDevice);
    if (st != hipSuccess) return fail(nullptr, BB_ERR_HIP, std::string("bb_gather_obs: ") + hipGetErrorString(st));
    s_dev = dev;
  }
  hipError_t st = launch_expand(d_board, d_hand, d_mask_bits, d_index, s_rows, n, d_x, d_mask_f32, nullptr,
                                (hipStream_t)stream);
  if (st != hipSuccess) return fail(nullptr, BB_ERR_HIP, std::string("bb_gather_obs: ") + hipGetErrorString(st));
  return BB_OK;
}

}  // extern "C"

namespace {
int bn_check(int32_t dtype, int32_t nhwc, int32_t N, int32_t C, int32_t HW) {
  if (dtype != 0 && dtype != 1) return fail(nullptr, BB_ERR_ARG, "bb_bn: dtype must be 0 (f32) or 1 (bf16)");
  if (nhwc != 0 && nhwc != 1) return fail(nullptr, BB_ERR_ARG, "bb_bn: layout must be 0 (NCHW) or 1 (NHWC)");
  if (N <= 0 || C <= 0 || HW <= 0) return fail(nullptr, BB_ERR_ARG, "bb_bn: empty tensor");
  const int esz = dtype == 1 ? 2 : 4;
  if (!nhwc && (HW * esz) % 16 != 0) return fail(nullptr, BB_ERR_ARG, "bb_bn: NCHW HW rows must be 16-byte multiples");
  if (nhwc && ((C * esz) % 16 != 0 || 256 % (C * esz / 16) != 0))
    return fail(nullptr, BB_ERR_ARG, "bb_bn: NHWC channel rows must be 16 B x a power of two <= 256");
  return BB_OK;
}
}  // namespace

extern "C" int64_t bb_bn_workspace_bytes(int32_t dtype, int32_t nhwc, int32_t N, int32_t C, int32_t HW) {
  if (bn_check(dtype, nhwc, N, C, HW) != BB_OK) return -1;
  return bn_workspace_bytes(dtype, nhwc, N, C, HW);
}

namespace {
int bn_forward_impl(const void* d_x, const void* d_res, int32_t dtype, int32_t nhwc, int32_t N, int32_t C, int32_t HW,
                    const float* d_pre_bias, const float* d_weight, const float* d_bias, float eps, int32_t relu,
                    double* d_ws, float* d_save_mean, float* d_save_invstd, float* d_running_mean,
                    float* d_running_var, float momentum, int64_t* d_num_batches_tracked, void* d_y, void* stream,
                    const char* what, const double* d_part = nullptr, int32_t nb_part = 0) {
  int rc = bn_check(dtype, nhwc, N, C, HW);
  if (rc != BB_OK) return rc;
  if (!d_x || !d_weight || !d_bias || !d_ws || !d_save_mean || !d_save_invstd || !d_y)
    return fail(nullptr, BB_ERR_ARG, std::string(what) + ": NULL argument");
  if (reinterpret_cast<uintptr_t>(d_ws) % 16 != 0) return fail(nullptr, BB_ERR_ARG, "bb_bn: d_ws must be 16-byte aligned");
  if (d_res && reinterpret_cast<uintptr_t>(d_res) % 16 != 0)
    return fail(nullptr, BB_ERR_ARG, "bb_bn: d_res must be 16-byte aligned");
  hipError_t st = launch_bn_forward(d_x, d_res, dtype, nhwc, N, C, HW, d_pre_bias, d_weight, d_bias, eps, relu, d_ws,
                                    d_save_mean, d_save_invstd, d_running_mean, d_running_var, momentum,
                                    d_num_batches_tracked, d_y, (hipStream_t)stream, d_part, nb_part);
  if (st != hipSuccess) return hip_fail(nullptr, st, what);
  return BB_OK;
}
}  // namespace

extern "C" int bb_bn_forward_part(const void* d_x, const void* d_res, int32_t dtype, int32_t nhwc, int32_t N,
                                  int32_t C, int32_t HW, const float* d_pre_bias, const float* d_weight,
                                  const float* d_bias, float eps, int32_t relu, double* d_ws, float* d_save_mean,
                                  float* d_save_invstd, float* d_running_mean, float* d_running_var, float momentum,
                                  int64_t* d_num_batches_tracked, void* d_y, const double* d_part, int32_t nb_part,
                                  void* stream) {
  if (!d_part || nb_part <= 0) return fail(nullptr, BB_ERR_ARG, "bb_bn_forward_part: no statistics partials");
  return bn_forward_impl(d_x, d_res, dtype, nhwc, N, C, HW, d_pre_bias, d_weight, d_bias, eps, relu, d_ws,
                         d_save_mean, d_save_invstd, d_running_mean, d_running_var, momentum, d_num_batches_tracked,
                         d_y, stream, "bb_bn_forward_part", d_part, nb_part);
}

extern "C" int bb_bn_forward(const void* d_x, int32_t dtype, int32_t nhwc, int32_t N, int32_t C, int32_t HW,
                             const float* d_pre_bias, const float* d_weight, const float* d_bias, float eps,
                             int32_t relu, double* d_ws, float* d_save_mean, float* d_save_invstd,
                             float* d_running_mean, float* d_running_var, float momentum,
                             int64_t* d_num_batches_tracked, void* d_y, void* stream) {
  return bn_forward_impl(d_x, nullptr, dtype, nhwc, N, C, HW, d_pre_bias, d_weight, d_bias, eps, relu, d_ws,
                         d_save_mean, d_save_invstd, d_running_mean, d_running_var, momentum, d_num_batches_tracked,
                         d_y, stream, "bb_bn_forward");
}

extern "C" int bb_bn_forward_res(const void* d_x, const void* d_res, int32_t dtype, int32_t nhwc, int32_t N,
                                 int32_t C, int32_t HW, const float* d_pre_bias, const float* d_weight,
                                 const float* d_bias, float eps, int32_t relu, double* d_ws, float* d_save_mean,
                                 float* d_save_invstd, float* d_running_mean, float* d_running_var, float momentum,
                                 int64_t* d_num_batches_tracked, void* d_y, void* stream) {
  if (!d_res) return fail(nullptr, BB_ERR_ARG, "bb_bn_forward_res: NULL residual");
  return bn_forward_impl(d_x, d_res, dtype, nhwc, N, C, HW, d_pre_bias, d_weight, d_bias, eps, relu, d_ws,
                         d_save_mean, d_save_invstd, d_running_mean, d_running_var, momentum, d_num_batches_tracked,
                         d_y, stream, "bb_bn_forward_res");
}

extern "C" int bb_bn_backward(const void* d_x, const void* d_dy, int32_t dtype, int32_t nhwc, int32_t N, int32_t C,
                              int32_t HW, const float* d_pre_bias, const float* d_weight, const float* d_bias,
                              const float* d_save_mean, const float* d_save_invstd, int32_t relu, double* d_ws,
                              void* d_dx, float* d_dweight, float* d_dbias, float* d_dpre_bias, void* stream) {
  int rc = bn_check(dtype, nhwc, N, C, HW);
  if (rc != BB_OK) return rc;
  if (!d_x || !d_dy || !d_weight || !d_bias || !d_save_mean || !d_save_invstd || !d_ws || !d_dx)
    return fail(nullptr, BB_ERR_ARG, "bb_bn_backward: NULL argument");
  if (reinterpret_cast<uintptr_t>(d_ws) % 16 != 0) return fail(nullptr, BB_ERR_ARG, "bb_bn: d_ws must be 16-byte aligned");
  hipError_t st = launch_bn_backward(d_x, d_dy, dtype, nhwc, N, C, HW, d_pre_bias, d_weight, d_bias, d_save_mean,
                                     d_save_invstd, relu, d_ws, d_dx, d_dweight, d_dbias, d_dpre_bias,
                                     (hipStream_t)stream);
  if (st != hipSuccess) return hip_fail(nullptr, st, "bb_bn_backward");
  return BB_OK;
}

extern "C" int bb_bn_backward_red(const void* d_x, const void* d_dy, int32_t dtype, int32_t nhwc, int32_t N, int32_t C,
                                  int32_t HW, const float* d_pre_bias, const float* d_weight, const float* d_bias,
                                  const float* d_save_mean, const float* d_save_invstd, int32_t relu, double* d_ws,
                                  void* d_dx, float* d_dweight, float* d_dbias, float* d_dpre_bias,
                                  const float* d_conv_ws, int32_t conv_chunks, int32_t conv_cin, int32_t conv_cout,
                                  int32_t conv_w_layout, float* d_conv_dw, void* stream) {
  int rc = bn_check(dtype, nhwc, N, C, HW);
  if (rc != BB_OK) return rc;
  if (!d_x || !d_dy || !d_weight || !d_bias || !d_save_mean || !d_save_invstd || !d_ws || !d_dx || !d_conv_ws ||
      !d_conv_dw || conv_chunks <= 0 || (conv_w_layout != 0 && conv_w_layout != 1) ||
      !conv3x3_supported(conv_cin, conv_cout))
    return fail(nullptr, BB_ERR_ARG, "bb_bn_backward_red: bad arguments");
  if (reinterpret_cast<uintptr_t>(d_ws) % 16 != 0) return fail(nullptr, BB_ERR_ARG, "bb_bn: d_ws must be 16-byte aligned");
  const WgradReduceJob job{d_conv_ws, conv_chunks, conv_cout, conv_cin, conv_w_layout, d_conv_dw};
  hipError_t st = launch_bn_backward(d_x, d_dy, dtype, nhwc, N, C, HW, d_pre_bias, d_weight, d_bias, d_save_mean,
                                     d_save_invstd, relu, d_ws, d_dx, d_dweight, d_dbias, d_dpre_bias,
                                     (hipStream_t)stream, nullptr, nullptr, &job);
  if (st != hipSuccess) return hip_fail(nullptr, st, "bb_bn_backward_red");
  return BB_OK;
}

extern "C" int bb_bn_backward_part(const void* d_x, const void* d_dy, int32_t dtype, int32_t nhwc, int32_t N,
                                   int32_t C, int32_t HW, const float* d_pre_bias, const float* d_weight,
                                   const float* d_bias, const float* d_save_mean, const float* d_save_invstd,
                                   int32_t relu, double* d_ws, void* d_dx, float* d_dweight, float* d_dbias,
                                   float* d_dpre_bias, const float* d_conv_ws, int32_t conv_chunks, int32_t conv_cin,
                                   int32_t conv_cout, int32_t conv_w_layout, float* d_conv_dw, const double* d_part,
                                   int32_t nb_part, void* stream) {
  int rc = bn_check(dtype, nhwc, N, C, HW);
  if (rc != BB_OK) return rc;
  if (!d_x || !d_dy || !d_weight || !d_bias || !d_save_mean || !d_save_invstd || !d_ws || !d_dx || !d_part ||
      nb_part <= 0)
    return fail(nullptr, BB_ERR_ARG, "bb_bn_backward_part: NULL argument");
  if (reinterpret_cast<uintptr_t>(d_ws) % 16 != 0) return fail(nullptr, BB_ERR_ARG, "bb_bn: d_ws must be 16-byte aligned");
  const bool red = d_conv_ws != nullptr;
  if (red && (!d_conv_dw || conv_chunks <= 0 || (conv_w_layout != 0 && conv_w_layout != 1) ||
              !conv3x3_supported(conv_cin, conv_cout)))
    return fail(nullptr, BB_ERR_ARG, "bb_bn_backward_part: bad convolution reduction arguments");
  const WgradReduceJob job{d_conv_ws, conv_chunks, conv_cout, conv_cin, conv_w_layout, d_conv_dw};
  hipError_t st = launch_bn_backward(d_x, d_dy, dtype, nhwc, N, C, HW, d_pre_bias, d_weight, d_bias, d_save_mean,
                                     d_save_invstd, relu, d_ws, d_dx, d_dweight, d_dbias, d_dpre_bias,
                                     (hipStream_t)stream, nullptr, nullptr, red ? &job : nullptr, d_part, nb_part);
  if (st != hipSuccess) return hip_fail(nullptr, st, "bb_bn_backward_part");
  return BB_OK;
}

extern "C" int bb_bn_backward_res(const void* d_x, const void* d_dy, const void* d_y, int32_t dtype, int32_t nhwc,
                                  int32_t N, int32_t C, int32_t HW, const float* d_pre_bias, const float* d_weight,
                                  const float* d_bias, const float* d_save_mean, const float* d_save_invstd,
                                  double* d_ws, void* d_dx, float* d_dweight, float* d_dbias, float* d_dpre_bias,
                                  void* d_gres, const float* d_conv_ws, int32_t conv_chunks, int32_t conv_cin,
                                  int32_t conv_cout, int32_t conv_w_layout, float* d_conv_dw, void* stream) {
  int rc = bn_check(dtype, nhwc, N, C, HW);
  if (rc != BB_OK) return rc;
  if (!d_x || !d_dy || !d_y || !d_weight || !d_bias || !d_save_mean || !d_save_invstd || !d_ws || !d_dx || !d_gres)
    return fail(nullptr, BB_ERR_ARG, "bb_bn_backward_res: NULL argument");
  if (reinterpret_cast<uintptr_t>(d_ws) % 16 != 0) return fail(nullptr, BB_ERR_ARG, "bb_bn: d_ws must be 16-byte aligned");
  const bool red = d_conv_ws != nullptr;
  if (red && (!d_conv_dw || conv_chunks <= 0 || (conv_w_layout != 0 && conv_w_layout != 1) ||
              !conv3x3_supported(conv_cin, conv_cout)))
    return fail(nullptr, BB_ERR_ARG, "bb_bn_backward_res: bad convolution reduction arguments");
  const WgradReduceJob job{d_conv_ws, conv_chunks, conv_cout, conv_cin, conv_w_layout, d_conv_dw};
  hipError_t st = launch_bn_backward(d_x, d_dy, dtype, nhwc, N, C, HW, d_pre_bias, d_weight, d_bias, d_save_mean,
                                     d_save_invstd, 0, d_ws, d_dx, d_dweight, d_dbias, d_dpre_bias, (hipStream_t)stream,
                                     d_y, d_gres, red ? &job : nullptr);
  if (st != hipSuccess) return hip_fail(nullptr, st, "bb_bn_backward_res");
  return BB_OK;
}

extern "C" int64_t bb_ppo_loss_workspace_bytes(int32_t B) {
  if (B <= 0) return -1;
  return ppo_loss_workspace_bytes(B);
}

namespace {
int loss_forward_impl(const void* d_logits, const void* d_values, int bf16, const float* d_mask,
                      const int64_t* d_actions, const float* d_old_logp, const float* d_adv, const float* d_ret,
                      int32_t B, float clip, float value_coef, float entropy_coef, double* d_ws, uint32_t* d_cnt,
                      float* d_stats, float* d_loss, void* stream, const char* what) {
  if (B <= 0 || !d_logits || !d_values || !d_mask || !d_actions || !d_old_logp || !d_adv || !d_ret || !d_ws ||
      !d_cnt || !d_stats)
    return fail(nullptr, BB_ERR_ARG, std::string(what) + ": bad arguments");
  hipError_t st = launch_ppo_loss_forward(d_logits, d_values, bf16, d_mask, d_actions, d_old_logp, d_adv, d_ret, B,
                                          clip, value_coef, entropy_coef, d_ws, d_cnt, d_stats, d_loss,
                                          (hipStream_t)stream);
  if (st != hipSuccess) return hip_fail(nullptr, st, what);
  return BB_OK;
}

int loss_backward_impl(const void* d_logits, const void* d_values, int bf16, const float* d_mask,
                       const int64_t* d_actions, const float* d_old_logp, const float* d_adv, const float* d_ret,
                       int32_t B, float clip, float value_coef, float entropy_coef, const float* d_grad_loss,
                       void* d_dlogits, void* d_dvalues, void* stream, const char* what) {
  if (B <= 0 || !d_logits || !d_values || !d_mask || !d_actions || !d_old_logp || !d_adv || !d_ret ||
      !d_grad_loss || !d_dlogits || !d_dvalues)
    return fail(nullptr, BB_ERR_ARG, std::string(what) + ": bad arguments");
  hipError_t st = launch_ppo_loss_backward(d_logits, d_values, bf16, d_mask, d_actions, d_old_logp, d_adv, d_ret, B,
                                           clip, value_coef, entropy_coef, d_grad_loss, d_dlogits, d_dvalues,
                                           (hipStream_t)stream);
  if (st != hipSuccess) return hip_fail(nullptr, st, what);
  return BB_OK;
}
}  // namespace

extern "C" int bb_ppo_loss_forward(const float* d_logits, const float* d_values, const float* d_mask,
                                   const int64_t* d_actions, const float* d_old_logp, const float* d_adv,
                                   const float* d_ret, int32_t B, float clip, float value_coef, float entropy_coef,
                                   double* d_ws, uint32_t* d_cnt, float* d_stats, float* d_loss, void* stream) {
  return loss_forward_impl(d_logits, d_values, 0, d_mask, d_actions, d_old_logp, d_adv, d_ret, B, clip, value_coef,
                           entropy_coef, d_ws, d_cnt, d_stats, d_loss, stream, "bb_ppo_loss_forward");
}

extern "C" int bb_ppo_loss_backward(const float* d_logits, const float* d_values, const float* d_mask,
                                    const int64_t* d_actions, const float* d_old_logp, const float* d_adv,
                                    const float* d_ret, int32_t B, float clip, float value_coef, float entropy_coef,
                                    const float* d_grad_loss, float* d_dlogits, float* d_dvalues, void* stream) {
  return loss_backward_impl(d_logits, d_values, 0, d_mask, d_actions, d_old_logp, d_adv, d_ret, B, clip, value_coef,
                            entropy_coef, d_grad_loss, d_dlogits, d_dvalues, stream, "bb_ppo_loss_backward");
}

extern "C" int bb_ppo_loss_forward_bf16(const void* d_logits, const void* d_values, const float* d_mask,
                                        const int64_t* d_actions, const float* d_old_logp, const float* d_adv,
                                        const float* d_ret, int32_t B, float clip, float value_coef,
                                        float entropy_coef, double* d_ws, uint32_t* d_cnt, float* d_stats,
                                        float* d_loss, void* stream) {
  return loss_forward_impl(d_logits, d_values, 1, d_mask, d_actions, d_old_logp, d_adv, d_ret, B, clip, value_coef,
                           entropy_coef, d_ws, d_cnt, d_stats, d_loss, stream, "bb_ppo_loss_forward_bf16");
}

extern "C" int bb_ppo_loss_fused(const void* d_logits, const void* d_values, int32_t bf16, const float* d_mask,
                                 const int64_t* d_actions, const float* d_old_logp, const float* d_adv,
                                 const float* d_ret, int32_t B, float clip, float value_coef, float entropy_coef,
                                 const float* d_grad_loss, void* d_dlogits, void* d_dvalues, double* d_ws,
                                 uint32_t* d_cnt, float* d_stats, float* d_loss, void* stream) {
  if (B <= 0 || !d_logits || !d_values || !d_mask || !d_actions || !d_old_logp || !d_adv || !d_ret || !d_grad_loss ||
      !d_dlogits || !d_dvalues || !d_ws || !d_cnt || !d_stats)
    return fail(nullptr, BB_ERR_ARG, "bb_ppo_loss_fused: bad arguments");
  hipError_t st = launch_ppo_loss_fused(d_logits, d_values, bf16 ? 1 : 0, d_mask, d_actions, d_old_logp, d_adv, d_ret,
                                        B, clip, value_coef, entropy_coef, d_grad_loss, d_dlogits, d_dvalues, d_ws,
                                        d_cnt, d_stats, d_loss, (hipStream_t)stream);
  if (st != hipSuccess) return hip_fail(nullptr, st, "bb_ppo_loss_fused");
  return BB_OK;
}

extern "C" int bb_ppo_loss_backward_bf16(const void* d_logits, const void* d_values, const float* d_mask,
                                         const int64_t* d_actions, const float* d_old_logp, const float* d_adv,
                                         const float* d_ret, int32_t B, float clip, float value_coef,
                                         float entropy_coef, const float* d_grad_loss, void* d_dlogits,
                                         void* d_dvalues, void* stream) {
  return loss_backward_impl(d_logits, d_values, 1, d_mask, d_actions, d_old_logp, d_adv, d_ret, B, clip, value_coef,
                            entropy_coef, d_grad_loss, d_dlogits, d_dvalues, stream, "bb_ppo_loss_backward_bf16");
}

namespace {
int conv_check(int32_t N, int32_t cin, int32_t cout, const char* what) {
  if (N <= 0) return fail(nullptr, BB_ERR_ARG, std::string(what) + ": empty batch");
  if (!conv3x3_supported(cin, cout))
    return fail(nullptr, BB_ERR_ARG, std::string(what) + ": channels must be 64 or 128 in and out");
  return BB_OK;
}
bool al16(const void* p) { return reinterpret_cast<uintptr_t>(p) % 16 == 0; }
}  // namespace

extern "C" int64_t bb_conv3x3_workspace_bytes(int32_t N, int32_t cin, int32_t cout) {
  if (conv_check(N, cin, cout, "bb_conv3x3_workspace_bytes") != BB_OK) return -1;
  return conv3x3_wgrad_workspace_bytes(N, cin, cout);
}

extern "C" int bb_conv3x3_prep(const float* d_w, int32_t cin, int32_t cout, int32_t w_layout, void* d_wf, void* d_wd,
                               void* stream) {
  int rc = conv_check(1, cin, cout, "bb_conv3x3_prep");
  if (rc != BB_OK) return rc;
  if (w_layout != 0 && w_layout != 1) return fail(nullptr, BB_ERR_ARG, "bb_conv3x3_prep: w_layout must be 0 or 1");
  if (!d_w || !d_wf || !d_wd) return fail(nullptr, BB_ERR_ARG, "bb_conv3x3_prep: NULL argument");
  if (!al16(d_wf) || !al16(d_wd)) return fail(nullptr, BB_ERR_ARG, "bb_conv3x3_prep: outputs must be 16-byte aligned");
  hipError_t st = launch_conv3x3_prep(d_w, cin, cout, w_layout, d_wf, d_wd, (hipStream_t)stream);
  if (st != hipSuccess) return hip_fail(nullptr, st, "bb_conv3x3_prep");
  return BB_OK;
}

extern "C" int bb_conv3x3_prep_multi(int32_t num_layers, const float* const* h_w, const int32_t* h_cin,
                                     const int32_t* h_cout, const int32_t* h_w_layout, void* const* h_wf,
                                     void* const* h_wd, void* stream) {
  if (num_layers <= 0 || num_layers > 16)
    return fail(nullptr, BB_ERR_ARG, "bb_conv3x3_prep_multi: 1 to 16 layers");
  if (!h_w || !h_cin || !h_cout || !h_w_layout || !h_wf || !h_wd)
    return fail(nullptr, BB_ERR_ARG, "bb_conv3x3_prep_multi: NULL argument");
  for (int l = 0; l < num_layers; ++l)
    if (!al16(h_wf[l]) || !al16(h_wd[l]))
      return fail(nullptr, BB_ERR_ARG, "bb_conv3x3_prep_multi: outputs must be 16-byte aligned");
  hipError_t st = launch_conv3x3_prep_multi(num_layers, h_w, h_cin, h_cout, h_w_layout, h_wf, h_wd,
                                            (hipStream_t)stream);
  if (st == hipErrorInvalidValue)
    return fail(nullptr, BB_ERR_ARG, "bb_conv3x3_prep_multi: NULL weight/output, channels not 64/128 or bad layout");
  if (st != hipSuccess) return hip_fail(nullptr, st, "bb_conv3x3_prep_multi");
  return BB_OK;
}

extern "C" int bb_conv3x3_forward(const void* d_x, const void* d_w, int32_t N, int32_t cin, int32_t cout, void* d_y,
                                  void* stream) {
  int rc = conv_check(N, cin, cout, "bb_conv3x3_forward");
  if (rc != BB_OK) return rc;
  if (!d_x || !d_w || !d_y) return fail(nullptr, BB_ERR_ARG, "bb_conv3x3_forward: NULL argument");
  if (!al16(d_x) || !al16(d_w) || !al16(d_y))
    return fail(nullptr, BB_ERR_ARG, "bb_conv3x3_forward: tensors must be 16-byte aligned");
  hipError_t st = launch_conv3x3_forward(d_x, d_w, N, cin, cout, d_y, (hipStream_t)stream);
  if (st != hipSuccess) return hip_fail(nullptr, st, "bb_conv3x3_forward");
  return BB_OK;
}

extern "C" int32_t bb_conv3x3_stats_blocks(int32_t N, int32_t cout) {
  return (cout == 64 || cout == 128) ? conv3x3_stats_blocks(N, cout) : -1;
}

extern "C" int bb_conv3x3_forward_stats(const void* d_x, const void* d_w, int32_t N, int32_t cin, int32_t cout,
                                        void* d_y, double* d_part, void* stream) {
  int rc = conv_check(N, cin, cout, "bb_conv3x3_forward_stats");
  if (rc != BB_OK) return rc;
  if (!d_x || !d_w || !d_y || !d_part) return fail(nullptr, BB_ERR_ARG, "bb_conv3x3_forward_stats: NULL argument");
  if (!al16(d_x) || !al16(d_w) || !al16(d_y))
    return fail(nullptr, BB_ERR_ARG, "bb_conv3x3_forward_stats: tensors must be 16-byte aligned");
  const ConvStatsArgs sa{d_part, nullptr, nullptr, nullptr, nullptr, nullptr, 0};
  hipError_t st = launch_conv3x3_forward(d_x, d_w, N, cin, cout, d_y, (hipStream_t)stream, nullptr, &sa);
  if (st == hipErrorInvalidValue)
    return fail(nullptr, BB_ERR_ARG, "bb_conv3x3_forward_stats: not available in this (variant) build");
  if (st != hipSuccess) return hip_fail(nullptr, st, "bb_conv3x3_forward_stats");
  return BB_OK;
}

extern "C" int bb_conv3x3_forward_bstats(const void* d_x, const void* d_w, int32_t N, int32_t cin, int32_t cout,
                                         void* d_y, const void* d_bn_x, const float* d_mean, const float* d_invstd,
                                         const float* d_weight, const float* d_bias, int32_t relu, double* d_part,
                                         void* stream) {
  int rc = conv_check(N, cin, cout, "bb_conv3x3_forward_bstats");
  if (rc != BB_OK) return rc;
  if (!d_x || !d_w || !d_y || !d_part || !d_bn_x || !d_mean || !d_invstd || !d_weight || !d_bias)
    return fail(nullptr, BB_ERR_ARG, "bb_conv3x3_forward_bstats: NULL argument");
  if (!al16(d_x) || !al16(d_w) || !al16(d_y) || !al16(d_bn_x))
    return fail(nullptr, BB_ERR_ARG, "bb_conv3x3_forward_bstats: tensors must be 16-byte aligned");
  const ConvStatsArgs sa{d_part, (const uint16_t*)d_bn_x, d_mean, d_invstd, d_weight, d_bias, relu ? 1 : 0};
  hipError_t st = launch_conv3x3_forward(d_x, d_w, N, cin, cout, d_y, (hipStream_t)stream, nullptr, &sa);
  if (st == hipErrorInvalidValue)
    return fail(nullptr, BB_ERR_ARG, "bb_conv3x3_forward_bstats: not available in this (variant) build");
  if (st != hipSuccess) return hip_fail(nullptr, st, "bb_conv3x3_forward_bstats");
  return BB_OK;
}

extern "C" int bb_conv3x3_forward_add(const void* d_x, const void* d_w, int32_t N, int32_t cin, int32_t cout,
                                      const void* d_add, void* d_y, void* stream) {
  int rc = conv_check(N, cin, cout, "bb_conv3x3_forward_add");
  if (rc != BB_OK) return rc;
  if (!d_x || !d_w || !d_y || !d_add) return fail(nullptr, BB_ERR_ARG, "bb_conv3x3_forward_add: NULL argument");
  if (!al16(d_x) || !al16(d_w) || !al16(d_y) || !al16(d_add))
    return fail(nullptr, BB_ERR_ARG, "bb_conv3x3_forward_add: tensors must be 16-byte aligned");
  hipError_t st = launch_conv3x3_forward(d_x, d_w, N, cin, cout, d_y, (hipStream_t)stream, d_add);
  if (st == hipErrorInvalidValue)
    return fail(nullptr, BB_ERR_ARG, "bb_conv3x3_forward_add: not available in this (variant) build");
  if (st != hipSuccess) return hip_fail(nullptr, st, "bb_conv3x3_forward_add");
  return BB_OK;
}

extern "C" int bb_conv3x3_wgrad(const void* d_x, const void* d_dy, int32_t N, int32_t cin, int32_t cout, float* d_ws,
                                int32_t w_layout, float* d_dw, void* stream) {
  int rc = conv_check(N, cin, cout, "bb_conv3x3_wgrad");
  if (rc != BB_OK) return rc;
  if (w_layout != 0 && w_layout != 1) return fail(nullptr, BB_ERR_ARG, "bb_conv3x3_wgrad: w_layout must be 0 or 1");
  if (!d_x || !d_dy || !d_ws || !d_dw) return fail(nullptr, BB_ERR_ARG, "bb_conv3x3_wgrad: NULL argument");
  if (!al16(d_x) || !al16(d_dy)) return fail(nullptr, BB_ERR_ARG, "bb_conv3x3_wgrad: tensors must be 16-byte aligned");
  hipError_t st = launch_conv3x3_wgrad(d_x, d_dy, N, cin, cout, d_ws, w_layout, d_dw, (hipStream_t)stream);
  if (st != hipSuccess) return hip_fail(nullptr, st, "bb_conv3x3_wgrad");
  return BB_OK;
}

extern "C" int32_t bb_conv3x3_wgrad_chunks(int32_t N, int32_t cin, int32_t cout) {
  if (conv_check(N, cin, cout, "bb_conv3x3_wgrad_chunks") != BB_OK) return -1;
  return conv3x3_wgrad_chunks_used(N, cin, cout);
}

extern "C" int bb_conv3x3_wgrad_partial(const void* d_x, const void* d_dy, int32_t N, int32_t cin, int32_t cout,
                                        float* d_ws, void* stream) {
  int rc = conv_check(N, cin, cout, "bb_conv3x3_wgrad_partial");
  if (rc != BB_OK) return rc;
  if (!d_x || !d_dy || !d_ws) return fail(nullptr, BB_ERR_ARG, "bb_conv3x3_wgrad_partial: NULL argument");
  if (!al16(d_x) || !al16(d_dy))
    return fail(nullptr, BB_ERR_ARG, "bb_conv3x3_wgrad_partial: tensors must be 16-byte aligned");
  hipError_t st = launch_conv3x3_wgrad_partial(d_x, d_dy, N, cin, cout, d_ws, (hipStream_t)stream);
  if (st != hipSuccess) return hip_fail(nullptr, st, "bb_conv3x3_wgrad_partial");
  return BB_OK;
}

extern "C" int bb_conv3x3_wgrad_reduce(const float* d_ws, int32_t chunks, int32_t cin, int32_t cout, int32_t w_layout,
                                       float* d_dw, void* stream) {
  int rc = conv_check(1, cin, cout, "bb_conv3x3_wgrad_reduce");
  if (rc != BB_OK) return rc;
  if (!d_ws || !d_dw || chunks <= 0 || (w_layout != 0 && w_layout != 1))
    return fail(nullptr, BB_ERR_ARG, "bb_conv3x3_wgrad_reduce: bad arguments");
  hipError_t st = launch_conv3x3_wgrad_reduce(d_ws, chunks, cin, cout, w_layout, d_dw, (hipStream_t)stream);
  if (st != hipSuccess) return hip_fail(nullptr, st, "bb_conv3x3_wgrad_reduce");
  return BB_OK;
}

extern "C" int bb_conv3x3_f32_prep(const float* d_w, int32_t cin, int32_t cout, int32_t w_layout, float* d_wf,
                                   float* d_wd, void* stream) {
  if (!conv3x3_f32_supported(cin, cout))
    return fail(nullptr, BB_ERR_ARG, "bb_conv3x3_f32_prep: (cin, cout) must be (128, 128), (64, 128) or (128, 64)");
  if (w_layout != 0 && w_layout != 1) return fail(nullptr, BB_ERR_ARG, "bb_conv3x3_f32_prep: w_layout must be 0 or 1");
  if (!d_w || (!d_wf && !d_wd)) return fail(nullptr, BB_ERR_ARG, "bb_conv3x3_f32_prep: NULL argument");
  if (!al16(d_wf) || !al16(d_wd)) return fail(nullptr, BB_ERR_ARG, "bb_conv3x3_f32_prep: outputs must be 16-byte aligned");
  hipError_t st = launch_conv3x3_f32_prep(d_w, cin, cout, w_layout, d_wf, d_wd, (hipStream_t)stream);
  if (st != hipSuccess) return hip_fail(nullptr, st, "bb_conv3x3_f32_prep");
  return BB_OK;
}

extern "C" int bb_conv3x3_f32_forward(const float* d_x, const float* d_w, int32_t N, int32_t cin, int32_t cout,
                                      float* d_y, void* stream) {
  if (N <= 0) return fail(nullptr, BB_ERR_ARG, "bb_conv3x3_f32_forward: empty batch");
  if (!conv3x3_f32_supported(cin, cout))
    return fail(nullptr, BB_ERR_ARG, "bb_conv3x3_f32_forward: (cin, cout) must be (128, 128), (64, 128) or (128, 64)");
  if (!d_x || !d_w || !d_y) return fail(nullptr, BB_ERR_ARG, "bb_conv3x3_f32_forward: NULL argument");
  if (!al16(d_x) || !al16(d_w) || !al16(d_y))
    return fail(nullptr, BB_ERR_ARG, "bb_conv3x3_f32_forward: tensors must be 16-byte aligned");
  hipError_t st = launch_conv3x3_f32_forward(d_x, d_w, N, cin, cout, d_y, (hipStream_t)stream);
  if (st != hipSuccess) return hip_fail(nullptr, st, "bb_conv3x3_f32_forward");
  return BB_OK;
}

extern "C" int bb_linear_f32(const float* d_x, const float* d_w, const float* d_bias, int32_t M, int32_t N, int32_t K,
                             float* d_y, void* stream) {
  if (M <= 0 || N <= 0 || K <= 0 || N % 128 || K % 32)
    return fail(nullptr, BB_ERR_ARG, "bb_linear_f32: M, N, K must be positive, N % 128 == 0, K % 32 == 0");
  if (!d_x || !d_w || !d_y) return fail(nullptr, BB_ERR_ARG, "bb_linear_f32: NULL argument");
  if (!al16(d_x) || !al16(d_w) || !al16(d_y))
    return fail(nullptr, BB_ERR_ARG, "bb_linear_f32: tensors must be 16-byte aligned");
  hipError_t st = launch_linear_f32(d_x, d_w, d_bias, M, N, K, d_y, (hipStream_t)stream);
  if (st != hipSuccess) return hip_fail(nullptr, st, "bb_linear_f32");
  return BB_OK;
}

static_assert(BB_OPT_MAX_TENSORS == kOptMaxTensors, "bbvec.h / bb_env_internal.h tensor-table size");

extern "C" int64_t bb_adam_clip_workspace_bytes(int32_t num_tensors, const int64_t* h_numel) {
  if (num_tensors <= 0 || num_tensors > BB_OPT_MAX_TENSORS || !h_numel) return -1;
  return adam_clip_workspace_bytes(num_tensors, h_numel);
}

extern "C" int bb_adam_clip_step(int32_t num_tensors, float* const* h_param, float* const* h_grad,
                                 float* const* h_exp_avg, float* const* h_exp_avg_sq, float* const* h_step,
                                 const int64_t* h_numel, double lr, double beta1, double beta2, double eps,
                                 float max_norm, double* d_ws, float* d_total_norm, void* stream) {
  if (num_tensors <= 0 || num_tensors > BB_OPT_MAX_TENSORS)
    return fail(nullptr, BB_ERR_ARG, "bb_adam_clip_step: 1 to BB_OPT_MAX_TENSORS tensors");
  if (!h_param || !h_grad || !h_exp_avg || !h_exp_avg_sq || !h_step || !h_numel || !d_ws)
    return fail(nullptr, BB_ERR_ARG, "bb_adam_clip_step: NULL argument");
  if (!al16(d_ws)) return fail(nullptr, BB_ERR_ARG, "bb_adam_clip_step: d_ws must be 16-byte aligned");
  hipError_t st = launch_adam_clip(num_tensors, h_param, h_grad, h_exp_avg, h_exp_avg_sq, h_step, h_numel, lr, beta1,
                                   beta2, eps, max_norm, d_ws, d_total_norm, (hipStream_t)stream);
  if (st == hipErrorInvalidValue)
    return fail(nullptr, BB_ERR_ARG, "bb_adam_clip_step: empty tensor or NULL tensor pointer");
  if (st != hipSuccess) return hip_fail(nullptr, st, "bb_adam_clip_step");
  return BB_OK;
}

extern "C" int bb_cast_multi(int32_t num_tensors, int32_t dir, const void* const* h_src, void* const* h_dst,
                             const int64_t* h_numel, const int32_t* h_perm_c, const int32_t* h_perm_hw, void* stream) {
  if (num_tensors <= 0 || num_tensors > BB_OPT_MAX_TENSORS)
    return fail(nullptr, BB_ERR_ARG, "bb_cast_multi: 1 to BB_OPT_MAX_TENSORS tensors");
  if (dir != 0 && dir != 1) return fail(nullptr, BB_ERR_ARG, "bb_cast_multi: dir must be 0 (f32->bf16) or 1");
  if (!h_src || !h_dst || !h_numel) return fail(nullptr, BB_ERR_ARG, "bb_cast_multi: NULL argument");
  hipError_t st = launch_cast_multi(num_tensors, dir, h_src, h_dst, h_numel, h_perm_c, h_perm_hw, (hipStream_t)stream);
  if (st == hipErrorInvalidValue)
    return fail(nullptr, BB_ERR_ARG, "bb_cast_multi: empty tensor, NULL pointer or bad permutation");
  if (st != hipSuccess) return hip_fail(nullptr, st, "bb_cast_multi");
  return BB_OK;
}

extern "C" int bb_dropout_forward(void* d_y, int64_t n, float p, int64_t* d_rng, void* stream) {
  if (!d_y || !d_rng) return fail(nullptr, BB_ERR_ARG, "bb_dropout_forward: NULL argument");
  if (n <= 0 || n % 8) return fail(nullptr, BB_ERR_ARG, "bb_dropout_forward: n must be a positive multiple of 8");
  if (!(p > 0.f && p < 1.f)) return fail(nullptr, BB_ERR_ARG, "bb_dropout_forward: p must be in (0, 1)");
  hipError_t st = launch_dropout_fwd(d_y, n, p, d_rng, (hipStream_t)stream);
  if (st == hipErrorInvalidValue) return fail(nullptr, BB_ERR_ARG, "bb_dropout_forward: y must be 16-byte aligned");
  if (st != hipSuccess) return hip_fail(nullptr, st, "bb_dropout_forward");
  return BB_OK;
}

extern "C" int bb_linear_bgrad2(const void* d_dy, const void* d_dy2, int32_t split, const void* d_yd, int32_t rows,
                                int32_t cols, float scale, void* d_g, void* d_db, float* d_ws, uint32_t* d_cnt,
                                void* stream) {
  if (!d_dy || !d_dy2 || !d_yd || !d_g || !d_db || !d_ws || !d_cnt)
    return fail(nullptr, BB_ERR_ARG, "bb_linear_bgrad2: NULL argument");
  if (rows <= 0 || cols <= 0) return fail(nullptr, BB_ERR_ARG, "bb_linear_bgrad2: rows and cols must be positive");
  hipError_t st = launch_linear_bgrad(d_dy, d_yd, rows, cols, scale, d_g, d_db, d_ws, d_cnt, (hipStream_t)stream, d_dy2,
                                      split);
  if (st == hipErrorInvalidValue)
    return fail(nullptr, BB_ERR_ARG, "bb_linear_bgrad2: split and cols - split multiples of 8, 16-byte aligned rows");
  if (st != hipSuccess) return hip_fail(nullptr, st, "bb_linear_bgrad2");
  return BB_OK;
}

extern "C" int64_t bb_linear_bgrad_workspace_bytes(int32_t rows, int32_t cols) {
  return linear_bgrad_workspace_bytes(rows, cols);
}

extern "C" int32_t bb_linear_bgrad_counters(int32_t cols) { return linear_bgrad_counters(cols); }

extern "C" int bb_linear_bgrad(const void* d_dy, const void* d_yd, int32_t rows, int32_t cols, float scale, void* d_g,
                               void* d_db, float* d_ws, uint32_t* d_cnt, void* stream) {
  if (!d_dy || !d_db || (d_yd && !d_g) || !d_ws || !d_cnt)
    return fail(nullptr, BB_ERR_ARG, "bb_linear_bgrad: NULL argument");
  if (rows <= 0 || cols <= 0) return fail(nullptr, BB_ERR_ARG, "bb_linear_bgrad: rows and cols must be positive");
  hipError_t st = launch_linear_bgrad(d_dy, d_yd, rows, cols, scale, d_g, d_db, d_ws, d_cnt, (hipStream_t)stream);
  if (st != hipSuccess) return hip_fail(nullptr, st, "bb_linear_bgrad");
  return BB_OK;
}

extern "C" int64_t bb_conv_in_wgrad_workspace_bytes(int32_t N) { return conv_in_wgrad_workspace_bytes(N); }

extern "C" int bb_conv_in_forward(const float* d_x, int32_t x_nhwc, const float* d_w, int32_t wl, int32_t N, void* d_y,
                                  void* stream) {
  if (!d_x || !d_w || !d_y) return fail(nullptr, BB_ERR_ARG, "bb_conv_in_forward: NULL argument");
  if (N <= 0) return fail(nullptr, BB_ERR_ARG, "bb_conv_in_forward: N must be positive");
  hipError_t st = launch_conv_in_forward(d_x, x_nhwc, d_w, wl, N, d_y, (hipStream_t)stream);
  if (st == hipErrorInvalidValue)
    return fail(nullptr, BB_ERR_ARG, "bb_conv_in_forward: wl must be 0 or 1, x and y 16-byte aligned");
  if (st != hipSuccess) return hip_fail(nullptr, st, "bb_conv_in_forward");
  return BB_OK;
}

extern "C" int bb_conv_in_forward_prep(const float* d_x, int32_t x_nhwc, const float* d_w, int32_t wl, int32_t N,
                                       void* d_y, int32_t count, const float* const* h_w, const int32_t* h_cin,
                                       const int32_t* h_cout, const int32_t* h_w_layout, void* const* h_wf,
                                       void* const* h_wd, void* stream) {
  if (!d_x || !d_w || !d_y || !h_w || !h_cin || !h_cout || !h_w_layout || !h_wf || !h_wd)
    return fail(nullptr, BB_ERR_ARG, "bb_conv_in_forward_prep: NULL argument");
  if (N <= 0) return fail(nullptr, BB_ERR_ARG, "bb_conv_in_forward_prep: N must be positive");
  hipError_t st = launch_conv_in_forward_prep(d_x, x_nhwc, d_w, wl, N, d_y, count, h_w, h_cin, h_cout, h_w_layout, h_wf,
                                              h_wd, (hipStream_t)stream);
  if (st == hipErrorInvalidValue)
    return fail(nullptr, BB_ERR_ARG, "bb_conv_in_forward_prep: bad layout, alignment or prep table (1 to 16 layers)");
  if (st != hipSuccess) return hip_fail(nullptr, st, "bb_conv_in_forward_prep");
  return BB_OK;
}

extern "C" int bb_conv_in_wgrad(const float* d_x, int32_t x_nhwc, const void* d_dy, int32_t N, float* d_ws, int32_t wl,
                                float* d_dw, void* stream) {
  if (!d_x || !d_dy || !d_ws || !d_dw) return fail(nullptr, BB_ERR_ARG, "bb_conv_in_wgrad: NULL argument");
  if (N <= 0) return fail(nullptr, BB_ERR_ARG, "bb_conv_in_wgrad: N must be positive");
  hipError_t st = launch_conv_in_wgrad(d_x, x_nhwc, d_dy, N, d_ws, wl, d_dw, (hipStream_t)stream);
  if (st == hipErrorInvalidValue)
    return fail(nullptr, BB_ERR_ARG, "bb_conv_in_wgrad: wl must be 0 or 1, x and dy 16-byte aligned");
  if (st != hipSuccess) return hip_fail(nullptr, st, "bb_conv_in_wgrad");
  return BB_OK;
}

extern "C" int64_t bb_linear_wgrad_workspace_bytes(int32_t rows, int32_t N, int32_t K) {
  return linear_wgrad_workspace_bytes(rows, N, K);
}

extern "C" int32_t bb_linear_wgrad_counters(int32_t N, int32_t K) { return linear_wgrad_counters(N, K); }

extern "C" int bb_linear_wgrad(const void* d_g, const void* d_x, int32_t rows, int32_t N, int32_t K, int32_t ldx,
                               void* d_dw, float* d_ws, uint32_t* d_cnt, void* stream) {
  if (!d_g || !d_x || !d_dw || !d_ws || !d_cnt) return fail(nullptr, BB_ERR_ARG, "bb_linear_wgrad: NULL argument");
  hipError_t st = launch_linear_wgrad(d_g, d_x, rows, N, K, ldx, d_dw, d_ws, d_cnt, (hipStream_t)stream);
  if (st == hipErrorInvalidValue)
    return fail(nullptr, BB_ERR_ARG,
                "bb_linear_wgrad: 0 < rows <= 16384, N and K multiples of 32, ldx >= K a multiple of 8, aligned rows");
  if (st != hipSuccess) return hip_fail(nullptr, st, "bb_linear_wgrad");
  return BB_OK;
}

extern "C" int64_t bb_linear_n1_workspace_bytes(int32_t rows, int32_t K) { return linear_n1_workspace_bytes(rows, K); }

extern "C" int32_t bb_linear_n1_counters(int32_t K) { return linear_n1_counters(K); }

extern "C" int bb_linear_n1_forward(const void* d_x, const void* d_w, const void* d_b, int32_t rows, int32_t K, int32_t ldx,
                                    void* d_y, void* stream) {
  hipError_t st = launch_linear_n1_forward(d_x, d_w, d_b, rows, K, ldx, d_y, (hipStream_t)stream);
  if (st == hipErrorInvalidValue)
    return fail(nullptr, BB_ERR_ARG,
                "bb_linear_n1_forward: rows > 0, K and ldx >= K multiples of 8, x / w non-NULL and aligned");
  if (st != hipSuccess) return hip_fail(nullptr, st, "bb_linear_n1_forward");
  return BB_OK;
}

extern "C" int bb_linear_n1_backward(const void* d_gy, const void* d_x, const void* d_w, int32_t rows, int32_t K,
                                     int32_t ldx, void* d_dx, void* d_dw, void* d_db, float* d_ws, uint32_t* d_cnt,
                                     void* stream) {
  hipError_t st =
      launch_linear_n1_backward(d_gy, d_x, d_w, rows, K, ldx, d_dx, d_dw, d_db, d_ws, d_cnt, (hipStream_t)stream);
  if (st == hipErrorInvalidValue)
    return fail(nullptr, BB_ERR_ARG,
                "bb_linear_n1_backward: rows > 0, K and ldx >= K multiples of 8, aligned non-NULL buffers");
  if (st != hipSuccess) return hip_fail(nullptr, st, "bb_linear_n1_backward");
  return BB_OK;
}
