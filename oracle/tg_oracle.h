/* tg_oracle.h — CPU restatement of the reference Treasure Game step path.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the parity oracle: only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it, and only as the checker / CPU baseline.  The
 * product path (gym-treasure-game_amd/, libtg_amd.so) never links or calls it.
 *
 * Pinned against golden vectors generated from the unmodified reference in the build
 * container (tests/golden/make_golden.py): CPython MT19937 KATs, full trajectories (uniform,
 * masked, auto-reset), 4096-env rolling hashes and 10k reset states.
 */
#ifndef TG_ORACLE_H
#define TG_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct tgo_level tgo_level;
typedef struct tgo_env tgo_env;

/* --- CPython `random` restatement (F1 KATs) ------------------------------------------- */
void tgo_rng_words(uint64_t seed, int n, uint32_t *out);     /* getrandbits(32) x n        */
void tgo_rng_random(uint64_t seed, int n, double *out);      /* random() x n               */
void tgo_rng_uniform5(uint64_t seed, double *out);           /* the 5 uniform() KAT calls  */
void tgo_rng_gauss(uint64_t seed, int pairs, double *out);   /* gauss(0,2), gauss(0,48/36) */

/* --- level ------------------------------------------------------------------------------ */
tgo_level *tgo_level_parse(const char *domain, const char *objects, const char *interactions);
void tgo_level_free(tgo_level *lv);

/* --- single env (reference semantics; env == random.seed(seed); TreasureGame(); reset()) - */
size_t tgo_env_size(void);
tgo_env *tgo_env_new(const tgo_level *lv, uint64_t seed, double obs[9]);
void tgo_env_free(tgo_env *e);
/* step(a): returns 0, or -1 for an out-of-range action (the reference raises IndexError).
 * Python list indexing: a in [-9, -1] wraps. */
int tgo_step(tgo_env *e, int action, double obs[9], int32_t *reward, uint8_t *valid,
             uint8_t *done);
void tgo_reset(tgo_env *e, double obs[9]);
unsigned tgo_mask(tgo_env *e);
uint64_t tgo_draws(const tgo_env *e);
int64_t tgo_ticks(const tgo_env *e);
/* internal state: px, py, jump_ticker, doors, handles, bolt, key cx, cy, gold cx, cy,
 * facing_right, total_actions (same columns as the golden `internal` arrays) */
void tgo_internal(const tgo_env *e, int32_t out[12]);
/* the 6 collision predicates of IM/:232-288 at an arbitrary pixel position / door state
 * (bit order: up_clear, can_go_up, can_go_down, can_go_left, can_go_right, can_fall) */
unsigned tgo_predicates(tgo_env *e, int px, int py, unsigned door_bits);
/* the same over the pixel box [x0,x1) x [y0,y1), row-major u8 */
void tgo_predicate_table(tgo_env *e, int x0, int x1, int y0, int y1, unsigned door_bits,
                         uint8_t *out);

/* --- batched driver (the CPU baseline and the parity generator) ------------------------- */
/* Runs envs g in [g0, g0+n), env g seeded seed_base+g, for `steps` env-steps with the
 * counter-hash action stream (policy 0 = uniform over 0..8, 1 = masked-uniform).
 * Any output pointer may be NULL.  Layouts are env-major: obs [n][steps+1][9] (t=0 is the
 * reset obs), reward/valid/done [n][steps+1], final_obs [n][steps+1][9] (pre-reset obs of
 * an auto-reset step, else == obs), hash/draws/ticks [n].  Returns 0 or -1. */
int tgo_run(const tgo_level *lv, uint64_t seed_base, int64_t g0, int64_t n, int steps,
            uint64_t action_seed, int policy, int autoreset, double *obs, int32_t *reward,
            uint8_t *valid, uint8_t *done, double *final_obs, uint64_t *hash, int64_t *draws,
            int64_t *ticks, int nthreads);

/* action stream + record hash shared with tests/golden/make_golden.py and the device code */
int tgo_run_episodes(const tgo_level *lv, uint64_t seed_base, int64_t g0, int64_t n, int steps,
                     uint64_t action_seed, int policy, int t_from, int64_t *count,
                     uint64_t *digest, int nthreads);
uint64_t tgo_sm64(uint64_t x);
uint64_t tgo_action_hash(uint64_t a0, uint64_t g, uint64_t t);
int tgo_pick_action(uint64_t a0, uint64_t g, uint64_t t, int masked, unsigned mask);
uint64_t tgo_rec_hash(uint64_t h, const double obs[9], int32_t reward, int valid, int done);

/* --- renderer (TG/:98-105 render('rgb_array') -> DR/ draw_domain); PARITY UNPINNED -------- */
/* sprites_rgba: TGO_SPR_COUNT (24) RGBA8 images of sw x sh in include/tg_amd.h TG_SPR_* order.
 * rgb: [H*48][W*48][3].  Returns 0, 1 (libm watch: a handle end point within 1e-9 of an
 * integer) or -1 (a handle shaft leaving the surface: unsupported). */
int tgo_render(const tgo_env *e, const uint8_t *sprites_rgba, int sw, int sh, uint8_t *rgb);
int tgo_run_render(const tgo_level *lv, uint64_t seed_base, const int64_t *envs, int64_t n,
                   int steps, uint64_t action_seed, int policy, int autoreset,
                   const uint8_t *sprites_rgba, int sw, int sh, uint8_t *frames, int nthreads);
/* Random(seed).choice over a sequence of length n, `count` times (DR/:83-86) */
void tgo_choice_seq(uint64_t seed, int n, int count, int32_t *out);

#ifdef __cplusplus
}
#endif
#endif
