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
 *   tg_render          TreasureGame.render('rgb_array')  treasure_game.py:98-105
 *                        -> _TreasureGameDrawer.draw_domain _treasure_game_impl/
 *                           _treasure_game_drawer.py:136-163, draw_object :238-269
 *                      (ObservationWrapper, treasure_game.py:38-51, renders every reset/step)
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
#define TG_ERR_RENDER (1u << 28)   /* render: a handle shaft end point within 1e-9 of an int()
                                      boundary (libm watch), or a shaft off the screen */
#define TG_ERR_WINDOW (1u << 29)  /* a lane drew past its staged draw codes (a bound broken: bug) */
#define TG_ERR_FLOW (1u << 30)    /* TG_MODE_FLOW: a k_flow wait ran past its 4-s bound (a bug; the
                                      launch ended early, its results are not valid) */

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

/* A Python-level random stream's state, as random.getstate() holds it (CPython random.py
 * getstate: (3, tuple of 624 MT19937 words + index, gauss_next)): the reference's envs all draw
 * from the process-global `random` (_treasure_game_impl.py:2, _objects.py:9). */
typedef struct {
  uint32_t mt[624];   /* the generation CPython's genrand_uint32 reads */
  uint32_t index;     /* its next word, 0..624 (624: twist before the next word) */
  uint32_t has_gauss; /* gauss_next is not None */
  double gauss_next;
} tg_pystate;

/* Counters accumulated over all tg_step calls since creation / tg_stats_reset. */
typedef struct {
  int64_t steps;        /* env-steps (one per env per tg_step) */
  int64_t valid_steps;  /* steps whose option could run (reward not None) */
  int64_t ticks;        /* primitive ticks (_TreasureGameImpl.step calls) */
  int64_t draws;        /* random() draws (2 MT words each) */
  int64_t episodes;     /* completed episodes (auto-reset) */
  int64_t episodes_dropped; /* records lost because the queue (max(4N, 65536)) was full */
  int64_t launches;     /* step-kernel launches */
  double kernel_ms;     /* summed kernel time of the timed step launches (tg_set_timing): each
                           kernel's span from its first wave's start to its last wave's end, by
                           in-kernel s_memrealtime stamps (100 MHz); nothing goes on the stream */
  int64_t regens;       /* MT19937 generations regenerated by the step kernels (624 words +
                           312 random() values each) */
  int64_t wave_ticks;   /* sum over the tick loops' wavefronts of their longest lane's ticks:
                           lane efficiency = ticks / (64 * wave_ticks) (an upper bound for the
                           go loops, whose lanes may also wait for the others' plain ticks) */
  int64_t timed_launches; /* launches timed (tg_set_timing) */
  double run_ms;        /* of kernel_ms, the second kernel (k_run in the compact mode; the single
                           kernel of the direct launches) */
  double regen_ms;      /* summed span of the k_regen launches while timing is on */
  int64_t regen_timed;  /* k_regen launches timed (while tg_set_timing is on) */
  int64_t regen_launches; /* k_regen launches (deferred MT regenerations, tg_regenerate) */
  double classify_ms;   /* of kernel_ms, k_classify */
} tg_stats;

/* Create N envs on `device`: env i is `random.seed(seed_base + global_offset + i);
 * TreasureGame()` (the constructor consumes 4 draws; call tg_reset for env.reset(), as with
 * the reference; seed_base + global_offset + N - 1 must not exceed 2^64 - 1).  Level text in
 * the reference's file formats (domain.txt,
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

/* step(action) of a 1-env handle, for the N=1 drop-in (TreasureGame.step, TG/:91-96), no
 * auto-reset (as the reference).  Outputs are HOST pointers: obs f64 [9], reward, valid, done.
 * By default (tg_set_serve) the call is served by a one-wave kernel resident on the device
 * (k_serve1) that polls a mailbox in pinned host memory: the call posts the action, spins on
 * the answer and returns the row the kernel wrote into pinned host memory -- no launch and no
 * synchronisation per call.  The server is launched by the first such call (after the work
 * queued on `stream`), stopped by any other call on the handle, and leaves by itself after
 * TG_SERVE_IDLE_US (default 500) microseconds without a command.  With serving off: one launch
 * on `stream` and one synchronisation of it. */
int tg_step1(tg_batch *h, int32_t action, double *obs, int32_t *reward, uint8_t *valid,
             uint8_t *done, void *stream);

/* The N = 1 calls (tg_step1, tg_step1_py, tg_reset1_py) through the resident server (on != 0,
 * the default unless TG_SERVE=0 at tg_create) or one launch + synchronisation each (0).  Stops
 * a running server.  Results are identical either way. */
int tg_set_serve(tg_batch *h, int on);

/* The N=1 drop-in drawing from a caller-held Python random stream instead of the env's own
 * (TreasureGame with the reference's module-global random, IM/:2, OB/:9): `st` (host memory)
 * is read at the call and written back with the stream advanced by exactly the draws the
 * reference's call makes, any index (odd ones too) and gauss_next included.  Served as tg_step1
 * (the resident server, or one launch and one synchronisation per call).
 *   tg_step1_py:  step(action) (TG/:91-96); outputs as tg_step1.
 *   tg_reset1_py: reset() (TG/:78-81, IM/:55-73: 2 uniform + 2 gauss), also the constructor's
 *                 build (IM/:31-53); obs f64 [9] host, may be NULL. */
int tg_step1_py(tg_batch *h, int32_t action, tg_pystate *st, double *obs, int32_t *reward,
                uint8_t *valid, uint8_t *done, void *stream);
int tg_reset1_py(tg_batch *h, tg_pystate *st, double *obs, void *stream);

/* tg_step1_py over a stream state kept elsewhere: `words` (624 uint32) and `index` (int32,
 * 0..624) are read at the call and written back advanced, in place -- for the N=1 drop-in,
 * the words and index of CPython's global random.Random object itself (Modules/_randommodule.c
 * keeps them as `int index; uint32_t state[624]`; the Python side checks the layout against
 * random.getstate() first), so a step costs no getstate / setstate.  A step draws no gauss, so
 * gauss_next is not an argument. */
int tg_step1_pywords(tg_batch *h, int32_t action, uint32_t *words, int32_t *index, double *obs,
                     int32_t *reward, uint8_t *valid, uint8_t *done, void *stream);

/* K steps in one call with the on-device synthetic policy (TG_POLICY_*): step t0 + s takes
 * the actions tg_policy_actions(action_seed, t0 + s) would give, evaluated inside the step's
 * first kernel (no action launch, no host round trip).  Outputs are step-major: actions (may
 * be NULL) int32 [K][N], obs (may be NULL) f64 [K][N][9], reward int32 [K][N], valid u8
 * [K][N], done u8 [K][N].  flags: TG_STEP_AUTORESET (episodes queue for tg_episodes).
 * Identical to K x (tg_policy_actions + tg_step).  The fused-rollout API of SURVEY §8f-3: the
 * reference has no batched or multi-step API (callers loop over TreasureGame.step, TG/:91-96). */
int tg_rollout(tg_batch *h, int32_t steps, uint64_t action_seed, int64_t t0, int policy,
               uint32_t flags, int32_t *actions, double *obs, int32_t *reward, uint8_t *valid,
               uint8_t *done, void *stream);

/* Step the batch as `groups` contiguous groups (1..16, each >= 4096 envs; 1 = off, the default)
 * in tg_rollout: each group's steps go on a stream of its own, forked from and joined back to
 * the caller's, so one group's latency-bound option loops overlap another's bandwidth-bound
 * passes.  Results are identical (the envs share nothing); counters and timing are unchanged
 * in meaning (timing samples group 0's kernels).  stagger != 0: group g + 1 starts after group
 * g's first k_classify.  Synchronises.  (No reference counterpart: batching is new.) */
int tg_set_groups(tg_batch *h, int32_t groups, int32_t stagger);

/* available_mask for every env: u16 [N], bit k == option k can run. */
int tg_available_mask(tg_batch *h, uint16_t *mask, void *stream);

/* available_mask of a 1-env handle (the N=1 drop-in's TreasureGame.available_mask, TG/:83-89)
 * into a HOST u16: served by the resident server like tg_step1 (so a mask read between steps
 * does not stop it), or one launch + synchronisation with serving off. */
int tg_available_mask1(tg_batch *h, uint16_t *mask, void *stream);

/* reset() of a 1-env handle on its own stream (the N=1 drop-in's TreasureGame(seed=s).reset(),
 * TG/:78-81) with the obs row into HOST memory (obs f64 [9], may be NULL): tg_reset of the one
 * env, served by the resident server like tg_step1, or one launch + synchronisation with
 * serving off. */
int tg_reset1(tg_batch *h, double *obs, void *stream);

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
/*   TG_MODE_FLOW: as TG_MODE_COMPACT for tg_step; tg_rollout runs up to 16 steps per launch of
 *     k_flow, in which each 64-env chunk is classified for step t + 1 as soon as its envs are
 *     done with step t (no batch-wide barrier between steps).  Results are
 *     identical to the other modes. */
#define TG_MODE_FLOW 2
/*   (Round 2's TG_MODE_ASYNC, all K steps of tg_rollout in one persistent launch, was exact
 *     but slower, 0.214 vs 0.142 ms per step, and was removed in round 3: DESIGN.md §9.1.) */
int tg_set_mode(tg_batch *h, int mode, int run_blocks);

/* HIP-event timing of every `every`-th step launch (tg_step, tg_rollout's launches; 0 = off):
 * three event records around a timed launch (start, after the first kernel, end), accumulated
 * into tg_stats.kernel_ms / run_ms / timed_launches.  An event record between two kernels costs
 * the stream a gap of several microseconds, so a benchmark samples (e.g. every 8th step). */
int tg_set_timing(tg_batch *h, int every);

/* Regenerate every stale MT half still queued now (k_regen).  The compact step lists the halves
 * its envs left stale and regenerates the lists of REGEN_STEPS (16) steps at once, so up to 15
 * steps' worth may be pending after a tg_step; results never depend on when this runs (a lane
 * that reaches a stale half regenerates it itself).  A timed loop calls it at its end so that it
 * contains the regeneration work of its own steps.  Asynchronous on `stream`. */
int tg_regenerate(tg_batch *h, void *stream);
/* Capacity of the completed-episode queue (default max(4N, 65536) records).  Records that
 * arrive while it is full are dropped and counted (tg_stats.episodes_dropped); the count is
 * clamped so that an undrained queue never overflows.  Reallocates the queue and discards
 * what it holds (synchronises). */
int tg_set_episode_capacity(tg_batch *h, int32_t cap);
/* The six collision predicates of _TreasureGameImpl (up_clear, can_go_up, can_go_down,
 * can_go_left, can_go_right, can_fall: _treasure_game_impl.py:232-288) evaluated BY THE DEVICE
 * at every pixel position of [x0, x1) x [y0, y1), doors closed per door_bits (bit i = door i of
 * the objects file): out u8 [(y1-y0)][(x1-x0)] (device), bit k = predicate k.  A check hook for
 * the device build of the cell-level probes against the reference's truth tables. */
int tg_predicate_table(tg_batch *h, int32_t x0, int32_t x1, int32_t y0, int32_t y1,
                       uint32_t door_bits, uint8_t *out, void *stream);
/* Counters (host, synchronises). */
int tg_get_stats(tg_batch *h, tg_stats *out);
int tg_stats_reset(tg_batch *h);
/* Resources of the step kernels as launched on this handle's device (no reference counterpart;
 * for the measurement's notes): kernel TG_KERNEL_*; out: workgroups per CU by the occupancy
 * API, VGPRs, SGPRs, static LDS bytes per 256-thread workgroup. */
#define TG_KERNEL_CLASSIFY 0 /* k_classify, uniform policy given as actions, auto-reset */
#define TG_KERNEL_RUN 1      /* k_run, auto-reset */
#define TG_KERNEL_REGEN 2    /* k_regen */
int tg_kernel_info(tg_batch *h, int kernel, int32_t *blocks_per_cu, int32_t *vgprs, int32_t *sgprs,
                   int32_t *lds_bytes);
/* Per-env MT19937 storage of this build (no reference counterpart; for sizing and for the
 * measurement's byte counts): ring_words = the word positions of the ring of pre-twisted
 * generations, stored_words = the words kept in HBM (the even generations), code_bytes = one
 * draw code per random() of the ring.  Any pointer may be NULL. */
int tg_mt_layout(int32_t *ring_words, int32_t *stored_words, int32_t *code_bytes);

/* Diagnostic (a timed region's fixed costs): `kernels` dependent launches of an
 * empty kernel of `blocks` 256-thread workgroups on `stream` (the platform's dispatch gap between
 * two dependent kernels, and an idle GPU's first dispatch).  No reference counterpart. */
int tg_probe_dispatch(int32_t kernels, int32_t blocks, void *stream);

/* Raw SoA state copy-out for checkpoints and tests (host buffers, synchronises; the MT
 * generations are gathered on the device and copied out in chunks of 64 Ki envs):
 * pos int32 [N][2], flags u32 [N], objs int32 [N][4] (key cx,cy, gold cx,cy),
 * ang f64 [N][2], mt u32 [N][624], mt_pos u32 [N], ep int32 [N][2] (auto-reset episode
 * return, length so far).  Any pointer may be NULL.
 * (mt, mt_pos) is the env's random.getstate() equivalent: the current MT19937 generation and
 * the index into it (CPython's state right after a twist, index 0..623). */
int tg_read_state(tg_batch *h, int32_t *pos, uint32_t *flags, int32_t *objs, double *ang,
                  uint32_t *mt, uint32_t *mt_pos, int32_t *ep);
/* Checkpoint restore, the inverse of tg_read_state (host buffers, synchronises): every env
 * continues bit-exactly from the given state.  All pointers but ep are required (ep NULL =
 * zeros); mt_pos must be even and <= 624 (this path's draws consume words in pairs; 624 =
 * CPython's "twist before the next draw"), i.e. any random.getstate() of the reference env
 * reached through step()/reset().  The episode queue and counters are not touched. */
int tg_write_state(tg_batch *h, const int32_t *pos, const uint32_t *flags, const int32_t *objs,
                   const double *ang, const uint32_t *mt, const uint32_t *mt_pos,
                   const int32_t *ep);

/* ---- render('rgb_array') -----------------------------------------------------------------
 * Sprite sheet: TG_SPR_COUNT RGBA8 images of sprite_w x sprite_h (the reference's PNGs decoded,
 * e.g. by PIL, in this order; the reference scales each to 48x48 at load, DR/:57-134). */
#define TG_SPR_BACKGROUND 0     /* 5 variants: sprites/background/background_{0..4}.png */
#define TG_SPR_WALL 5           /* 5 variants: sprites/wall/wall_{0..4}.png */
#define TG_SPR_FLOOR 10         /* 5 variants: sprites/floor/floor-{0..4}.png */
#define TG_SPR_LADDER 15        /* sprites/ladder.png */
#define TG_SPR_DOOR_CLOSED 16   /* sprites/closeddoor.png */
#define TG_SPR_DOOR_OPEN 17     /* sprites/open-door.png */
#define TG_SPR_KEY 18           /* sprites/key.png */
#define TG_SPR_GOLD 19          /* sprites/gold.png */
#define TG_SPR_BOLT_OPEN 20     /* sprites/bolt-open.png */
#define TG_SPR_BOLT_LOCKED 21   /* sprites/bolt-locked.png */
#define TG_SPR_HERO 22          /* sprites/hero.png */
#define TG_SPR_HANDLE_BASE 23   /* sprites/handle-base.png */
#define TG_SPR_COUNT 24

/* Build the renderer's static layer and sprite tables (HOST sprite pointer; synchronises).
 * Must precede tg_render; may be called again to change the sheet. */
int tg_render_init(tg_batch *h, const uint8_t *sprites_rgba, int32_t sprite_w, int32_t sprite_h);
/* Frame size in pixels: H*48 rows x W*48 columns (624 x 672 for the default level). */
int tg_frame_shape(const tg_batch *h, int32_t *height, int32_t *width);
/* render('rgb_array') of envs [first, first+count): rgb u8 [count][height][width][3] (device,
 * 16-B aligned), the screen of each env's current state (after auto-reset, the new episode's). */
int tg_render(tg_batch *h, int64_t first, int64_t count, uint8_t *rgb, void *stream);

const char *tg_last_error(void);
const char *tg_version(void);

#ifdef __cplusplus
}
#endif
#endif /* TG_AMD_H */
