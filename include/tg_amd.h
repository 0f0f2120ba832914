/* tg_amd.h — C ABI of the MI355X batched Treasure Game simulator (libtg_amd.so).
 *
 * This is the drop-in boundary for the reference env's hot path.  One handle owns a batch of
 * N independent envs resident in HBM (struct-of-arrays state + one CPython-compatible
 * MT19937 stream per env).  Env g of a handle created with (seed_base, global_offset) is
 * bit-identical to the reference env made by
 *     random.seed(seed_base + global_offset + g); env = TreasureGame()
 * and replays the reference's reset()/step()/available_mask on the same calls.
 *
 * Conventions
 *   - every buffer argument is a DEVICE pointer on the handle's device (caller-owned);
 *   - `stream` is a hipStream_t passed as void* (NULL = the default stream); every call is
 *     asynchronous on that stream unless documented otherwise, and calls on one handle must
 *     be serialised by the caller (one handle = one stream, not re-entrant);
 *   - functions return TG_OK (0) or a negative TG_E* code; tg_last_error() gives the text
 *     (thread-local);
 *   - no torch or HIP types appear here.
 *
 * Reference interfaces replaced (paths under gym_treasure_game/envs/ of the reference):
 *   tg_create          TreasureGame.__init__            treasure_game.py:63-76
 *   tg_reset           TreasureGame.reset               treasure_game.py:78-81
 *   tg_step            TreasureGame.step                treasure_game.py:91-96
 *                        -> _Option.run              _treasure_game_impl/_option.py:20-36
 *                        -> _TreasureGameImpl.step   _treasure_game_impl/_treasure_game_impl.py:290-359
 *   tg_available_mask  TreasureGame.available_mask      treasure_game.py:83-89
 *   obs layout         _TreasureGameImpl.get_state      _treasure_game_impl.py:368-378
 *   level text         the 3 level files read by        _treasure_game_impl.py:75-202
 */
#ifndef TG_AMD_H
#define TG_AMD_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TG_OK 0
#define TG_E_INVAL (-1)    /* bad argument / level */
#define TG_E_HIP (-2)      /* HIP runtime error */
#define TG_E_NOMEM (-3)    /* device allocation failed */
#define TG_E_NODEV (-4)    /* no usable gfx950 device */
#define TG_E_STATE (-5)    /* an env hit an error flag (see tg_errors) */

#define TG_OBS_DIM 9       /* playerx, playery, handle1.angle, handle2.angle, key.x, key.y,
                              bolt.locked, goldcoin.x, goldcoin.y (IM/:380-400) */
#define TG_NUM_ACTIONS 9   /* go_left, go_right, up_ladder, down_ladder, interact, down_left,
                              down_right, jump_left, jump_right (IM/:495) */

/* per-env error bits reported by tg_errors() */
#define TG_ERR_TICKCAP (1u << 24)  /* an option ran > 16384 ticks (the reference would loop) */
#define TG_ERR_BAG (1u << 25)      /* bag overflow */
#define TG_ERR_ACTION (1u << 26)   /* action outside [-9, 8]: the reference raises IndexError */
#define TG_ERR_NEARINT (1u << 27)  /* reset gauss within 1e-9 of an int() boundary (libm watch) */

/* step flags */
#define TG_STEP_AUTORESET 1u       /* reset() an env right after a step that returned done */

/* action policies of tg_policy_actions */
#define TG_POLICY_UNIFORM 0        /* a = h(action_seed, g, t) % 9 (action_space.sample stand-in) */
#define TG_POLICY_MASKED 1         /* k-th set bit of available_mask, k = h % popcount */

typedef struct tg_batch tg_batch;

/* Completed episode record written by an auto-reset step. */
typedef struct {
  int64_t env;      /* global env index (global_offset + local index) */
  int32_t ret;      /* sum of step rewards since the last reset (None counts 0) */
  int32_t len;      /* env-steps since the last reset */
} tg_episode;

/* Counters accumulated over all tg_step calls since creation / tg_stats_reset. */
typedef struct {
  int64_t steps;        /* env-steps (one per env per tg_step) */
  int64_t valid_steps;  /* steps whose option could run (reward not None) */
  int64_t ticks;        /* primitive ticks (_TreasureGameImpl.step calls) */
  int64_t draws;        /* random() draws (2 MT words each) */
  int64_t episodes;     /* completed episodes (auto-reset) */
  int64_t episodes_dropped; /* records lost because the queue (max(4N, 65536)) was full */
  int64_t launches;     /* step-kernel launches */
  double kernel_ms;     /* summed step-kernel time measured with HIP events (if enabled) */
} tg_stats;

/* Create N envs on `device`: env i is `random.seed(seed_base + global_offset + i);
 * TreasureGame()` (the constructor consumes 4 draws; call tg_reset for env.reset(), as with
 * the reference).  Level text in the reference's file formats (domain.txt,
 * domain-objects.txt, domain-interactions.txt); NULL for all three = the built-in default
 * level.  Synchronises. */
int tg_create(tg_batch **out, int64_t num_envs, uint64_t seed_base, int64_t global_offset,
              int device, const char *domain_txt, const char *objects_txt,
              const char *interactions_txt);
void tg_destroy(tg_batch *h);

int64_t tg_num_envs(const tg_batch *h);

/* reset(): all envs (mask == NULL) or those with mask[i] != 0; writes obs [N][9] f64 for
 * every env (current obs for the ones not reset).  obs may be NULL. */
int tg_reset(tg_batch *h, const uint8_t *mask, double *obs, void *stream);

/* step(a) for every env: actions int32 [N] in [-9, 8] (Python list indexing).  Outputs:
 * obs f64 [N][9], reward int32 [N] (0 when not valid), valid u8 [N] (0 == reward None),
 * done u8 [N].  flags: TG_STEP_AUTORESET; then final_obs (may be NULL) receives the pre-reset
 * obs of every env (== obs where no reset happened) and completed episodes are appended to
 * the handle's episode buffer (tg_episodes). */
int tg_step(tg_batch *h, const int32_t *actions, double *obs, int32_t *reward, uint8_t *valid,
            uint8_t *done, double *final_obs, uint32_t flags, void *stream);

/* available_mask for every env: u16 [N], bit k == option k can run. */
int tg_available_mask(tg_batch *h, uint16_t *mask, void *stream);

/* current observation of every env, f64 [N][9]. */
int tg_observe(tg_batch *h, double *obs, void *stream);

/* Synthetic action stream for step t (bench / parity): see TG_POLICY_*.  g is the GLOBAL env
 * index, so trajectories are independent of how the batch is sharded. */
int tg_policy_actions(tg_batch *h, uint64_t action_seed, int64_t t, int policy, int32_t *actions,
                      void *stream);

/* Moves up to `cap` completed-episode records (oldest first) to the device buffer `out` and
 * their number (int32) to the device word `count`; the rest stay queued for the next call.
 * Asynchronous (no host sync), so it can feed a per-step RCCL gather directly. */
int tg_episodes(tg_batch *h, tg_episode *out, int32_t *count, int32_t cap, void *stream);

/* OR of all per-env error bits (host, synchronises the handle's stream). */
int tg_errors(tg_batch *h, uint32_t *or_of_flags, void *stream);

/* Step implementation (both bit-identical):
 *   TG_MODE_COMPACT (default): k_classify finishes envs whose option cannot run and appends
 *     the rest to per-option worklists; k_run's waves run them in 64-env chunks,
 *     longest-option-first (run_blocks is reserved, pass 0).
 *   TG_MODE_DIRECT: one k_step lane per env runs its option in place. */
#define TG_MODE_DIRECT 0
#define TG_MODE_COMPACT 1
int tg_set_mode(tg_batch *h, int mode, int run_blocks);

/* Enable HIP-event timing of every tg_step (adds two event records per step; the measured
 * interval covers all of the step's kernels). */
int tg_set_timing(tg_batch *h, int enable);
/* Counters (host, synchronises). */
int tg_get_stats(tg_batch *h, tg_stats *out);
int tg_stats_reset(tg_batch *h);

/* Raw SoA state copy-out for checkpoints and tests (host buffers, synchronises):
 * pos int32 [N][2], flags u32 [N], objs int32 [N][4] (key cx,cy, gold cx,cy),
 * ang f64 [N][2], mt u32 [N][624], mt_pos u32 [N].  Any pointer may be NULL.
 * (mt, mt_pos) is the env's random.getstate() equivalent: the current MT19937 generation and
 * the index into it (CPython's state right after a twist, index 0..623). */
int tg_read_state(tg_batch *h, int32_t *pos, uint32_t *flags, int32_t *objs, double *ang,
                  uint32_t *mt, uint32_t *mt_pos);

const char *tg_last_error(void);
const char *tg_version(void);

#ifdef __cplusplus
}
#endif
#endif /* TG_AMD_H */
