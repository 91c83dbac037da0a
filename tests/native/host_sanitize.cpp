// Sanitizer driver for the host backend (csrc/bb_host.cpp, SURVEY.md section 5 "a -fsanitize=address
// build of the C++ CPU backend").  TEST INFRASTRUCTURE: built by tests/test_host_sanitize.py with
// -fsanitize=address,undefined together with the C oracle (oracle/bb_oracle.c, the checker), it drives
// every env entry point of include/bbvec.h -- create, seed (seeded and seed_value-None envs), reset,
// obs, the fused rollout, single steps with legal, illegal and out-of-range actions, info records,
// get_state / set_state, masked reset, destroy -- and compares each output with the oracle bit for bit.
// Any sanitizer report aborts the process; a mismatch exits 1.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "bbvec.h"

extern "C" {
typedef struct bbo_vec bbo_vec;
bbo_vec* bbo_create(int n, const uint64_t* seeds, const uint8_t* has_seed, const double* rewards, int autoreset);
void bbo_destroy(bbo_vec* v);
void bbo_reset(bbo_vec* v, int threads);
void bbo_step(bbo_vec* v, const int32_t* actions, float* reward, double* reward64, uint8_t* term, uint8_t* lines,
              uint8_t* invalid, uint64_t* mask, int threads);
void bbo_rollout(bbo_vec* v, int T, int32_t* act_io, uint64_t policy_seed, uint64_t policy_step0,
                 uint64_t env_offset, float* reward, uint8_t* term, uint8_t* lines, int32_t* actions,
                 uint64_t* mask, int threads);
void bbo_random_actions(const uint64_t* mask, int n, uint64_t seed, uint64_t step, uint64_t env_offset,
                        int32_t* out);
void bbo_state(const bbo_vec* v, uint64_t* board, uint32_t* hand, int64_t* score, int32_t* combo,
               int32_t* max_combo, int32_t* moves, int32_t* lines, int32_t* blocks, uint8_t* prev_holes,
               uint8_t* prev_center, uint64_t* rng, uint64_t* mask);
}

static int g_fail = 0;

template <typename T>
static void expect_eq(const char* what, const std::vector<T>& a, const std::vector<T>& b) {
  if (a.size() != b.size() || memcmp(a.data(), b.data(), a.size() * sizeof(T)) != 0) {
    size_t k = 0;
    while (k < a.size() && memcmp(&a[k], &b[k], sizeof(T)) == 0) ++k;
    fprintf(stderr, "MISMATCH %s at element %zu of %zu\n", what, k, a.size());
    g_fail = 1;
  }
}

static int ok(int rc, const char* what, bb_env* env) {
  if (rc != BB_OK) {
    fprintf(stderr, "%s failed (%d): %s\n", what, rc, bb_last_error(env));
    exit(2);
  }
  return rc;
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 517;
  const int T = argc > 2 ? atoi(argv[2]) : 160;
  const uint64_t kPolicy = 0xB10C;
  const bb_reward_cfg cfg = {1.0, 0.01, -1.0, -0.05, 0.02, 0.5, 0.001};  // block_blast_env.py:63-73

  // every third env has seed_value None: its stream continues across resets (engine.py:137-138); the
  // oracle starts it from default_rng(seed) as well, so the host gets those words as raw state
  std::vector<uint64_t> seeds(n), raw(4 * (size_t)n);
  std::vector<uint8_t> has(n);
  for (int i = 0; i < n; ++i) {
    seeds[i] = 42 + (uint64_t)i;
    has[i] = i % 3 == 2 ? 0 : 1;
    ok(bb_pcg64_seed(seeds[i], &raw[4 * (size_t)i]), "bb_pcg64_seed", nullptr);
  }
  bb_env* env = nullptr;
  ok(bb_create(n, 0, &cfg, 1, &env), "bb_create", nullptr);
  ok(bb_seed(env, seeds.data(), has.data(), raw.data()), "bb_seed", env);
  ok(bb_reset(env, nullptr, nullptr), "bb_reset", env);
  bbo_vec* v = bbo_create(n, seeds.data(), has.data(), nullptr, 1);
  bbo_reset(v, 0);

  // observations of the reset state
  std::vector<float> x((size_t)n * 256), mf((size_t)n * 192);
  std::vector<int8_t> mi((size_t)n * 192);
  std::vector<uint64_t> mb(3 * (size_t)n), mo(3 * (size_t)n);
  ok(bb_obs(env, x.data(), mi.data(), mf.data(), mb.data(), nullptr), "bb_obs", env);
  bbo_state(v, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
            mo.data());
  expect_eq("reset mask", mb, mo);

  // the fused rollout (bb_rollout) against the oracle's
  std::vector<int32_t> a0(n), a0o(n);
  ok(bb_random_actions(mb.data(), n, kPolicy, 0, 0, a0.data(), nullptr), "bb_random_actions", env);
  bbo_random_actions(mo.data(), n, kPolicy, 0, 0, a0o.data());
  expect_eq("first actions", a0, a0o);
  std::vector<float> rw((size_t)T * n), rwo((size_t)T * n);
  std::vector<uint8_t> tm((size_t)T * n), tmo((size_t)T * n), ln((size_t)T * n), lno((size_t)T * n);
  std::vector<int32_t> ac((size_t)T * n), aco((size_t)T * n), nx(n);
  std::vector<uint64_t> rm(3 * (size_t)T * n), rmo(3 * (size_t)T * n);
  bb_rollout_out ro{rw.data(), tm.data(), ln.data(), ac.data(), rm.data(), nx.data(), kPolicy, 0, 0};
  ok(bb_rollout(env, T, a0.data(), &ro, nullptr), "bb_rollout", env);
  ok(bb_sync(env, nullptr), "bb_sync", env);
  bbo_rollout(v, T, a0o.data(), kPolicy, 0, 0, rwo.data(), tmo.data(), lno.data(), aco.data(), rmo.data(), 0);
  expect_eq("rollout reward", rw, rwo);
  expect_eq("rollout terminated", tm, tmo);
  expect_eq("rollout lines", ln, lno);
  expect_eq("rollout actions", ac, aco);
  expect_eq("rollout mask", rm, rmo);
  expect_eq("rollout next action", nx, a0o);

  // single steps (bb_step): policy actions with illegal and out-of-range ones mixed in, fp64 reward, info
  std::vector<float> r1(n), r1o(n);
  std::vector<double> r64(n), r64o(n);
  std::vector<uint8_t> t1(n), t1o(n), l1(n), l1o(n);
  std::vector<bb_info> info(n);
  std::vector<int64_t> fs(n, -1);
  std::vector<int32_t> fm(n, -1), next(n);
  std::vector<int32_t> act = nx;
  for (int s = 0; s < 40; ++s) {
    for (int i = 0; i < n; ++i) {
      const int k = (i * 7 + s * 13) % 29;
      if (k == 0) act[i] = -1 - (i % 5);
      else if (k == 1) act[i] = 192 + i % 400;
      else if (k == 2) act[i] = (act[i] + 64) % 192;  // often an illegal slot / anchor
    }
    bb_step_out so{r1.data(), t1.data(), r64.data(), mb.data(), l1.data(), info.data(), next.data(), kPolicy,
                   (uint64_t)(T + s + 1), 0, fs.data(), fm.data()};
    ok(bb_step(env, act.data(), &so, nullptr), "bb_step", env);
    bbo_step(v, act.data(), r1o.data(), r64o.data(), t1o.data(), l1o.data(), nullptr, mo.data(), 0);
    expect_eq("step reward", r1, r1o);
    expect_eq("step reward f64", r64, r64o);
    expect_eq("step terminated", t1, t1o);
    expect_eq("step lines", l1, l1o);
    expect_eq("step mask", mb, mo);
    std::vector<int32_t> nxo(n);
    bbo_random_actions(mo.data(), n, kPolicy, (uint64_t)(T + s + 1), 0, nxo.data());
    expect_eq("step next action", next, nxo);
    act = next;
  }

  // packed state against the oracle's, then a set_state round trip and a masked reset
  std::vector<uint64_t> b(n), bo(n), rg(3 * (size_t)n), rgo(3 * (size_t)n);
  std::vector<uint32_t> h(n), ho(n);
  std::vector<int64_t> sc(n), sco(n);
  std::vector<int32_t> cb(n), cbo(n), mc(n), mco(n), mv(n), mvo(n), li(n), lio(n), bl(n), blo(n);
  std::vector<uint8_t> ph(n), pho(n), pc(n), pco(n);
  bb_state_view sv{b.data(), h.data(), sc.data(), cb.data(), mc.data(), mv.data(), li.data(), bl.data(),
                   ph.data(), pc.data(), rg.data()};
  ok(bb_get_state(env, &sv), "bb_get_state", env);
  bbo_state(v, bo.data(), ho.data(), sco.data(), cbo.data(), mco.data(), mvo.data(), lio.data(), blo.data(),
            pho.data(), pco.data(), rgo.data(), nullptr);
  expect_eq("state board", b, bo);
  expect_eq("state hand", h, ho);
  expect_eq("state score", sc, sco);
  expect_eq("state combo", cb, cbo);
  expect_eq("state max_combo", mc, mco);
  expect_eq("state moves", mv, mvo);
  expect_eq("state lines", li, lio);
  expect_eq("state blocks", bl, blo);
  expect_eq("state prev_holes", ph, pho);
  expect_eq("state prev_center", pc, pco);
  for (int i = 0; i < n; ++i)  // uinteger is meaningful only while has_uint32 (hand bit 22) is set
    if (!((h[i] >> 22) & 1u)) rg[3 * (size_t)i + 2] = rgo[3 * (size_t)i + 2] = 0;
  expect_eq("state rng", rg, rgo);
  ok(bb_set_state(env, &sv), "bb_set_state", env);
  std::vector<uint64_t> b2(n);
  bb_state_view sv2{b2.data(), nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                    nullptr};
  ok(bb_get_state(env, &sv2), "bb_get_state", env);
  expect_eq("set_state round trip", b2, b);
  std::vector<uint8_t> sel(n);
  for (int i = 0; i < n; ++i) sel[i] = (uint8_t)(i % 2);
  ok(bb_reset(env, sel.data(), nullptr), "bb_reset (masked)", env);
  ok(bb_get_state(env, &sv2), "bb_get_state", env);
  for (int i = 0; i < n; ++i)
    if ((sel[i] && b2[i] != 0) || (!sel[i] && b2[i] != b[i])) {
      fprintf(stderr, "MISMATCH masked reset at env %d\n", i);
      g_fail = 1;
      break;
    }

  // argument errors are reported, not crashes
  if (bb_step(env, nullptr, nullptr, nullptr) != BB_ERR_ARG || bb_rollout(env, -1, a0.data(), &ro, nullptr) != BB_ERR_ARG ||
      bb_create(0, 0, &cfg, 1, nullptr) != BB_ERR_ARG) {
    fprintf(stderr, "argument checks\n");
    g_fail = 1;
  }
  bb_destroy(env);
  bbo_destroy(v);
  if (g_fail) return 1;
  printf("host backend under sanitizers: %d envs, %d rollout steps + 40 steps, bit-exact vs the C oracle\n", n, T);
  return 0;
}
