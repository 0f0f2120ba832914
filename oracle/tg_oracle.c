/* tg_oracle.c — CPU restatement of the reference Treasure Game (TEST INFRASTRUCTURE ONLY).
 *
 * Header: see tg_oracle.h.  The product never links this file.  It restates the reference
 * structure literally (so that it is an independent check of the GPU kernel's cell-level
 * collapse):
 *   - collision predicates loop over the same pixel probes as the reference (IM/:232-288);
 *     the pixel map is stored at cell granularity, which is exact because build_map repeats
 *     every character 48x48 (IM/:204-216) and door.update_map rewrites whole cells
 *     (OB/:246-253);
 *   - objects keep the reference's object list, trigger lists and the recursive
 *     process_trigger cascade with its re-entrancy guard (OB/:65-94);
 *   - the bag is the reference's Python list (IM/:44, 350-354, 434-439);
 *   - randomness is a restatement of CPython 3.10's `random` (MT19937 in _randommodule.c,
 *     random/uniform/gauss in Lib/random.py) with glibc libm, exactly what the reference calls.
 * Citation prefixes: TG/ treasure_game.py, IM/ _treasure_game_impl.py, OB/ _objects.py,
 * MO/ _move_options.py, OP/ _option.py (all under gym_treasure_game/envs/).
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off -fopenmp); never -ffast-math.
 */
#include "tg_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ======================================================================================
 * CPython random (Modules/_randommodule.c + Lib/random.py, CPython 3.10)
 * ====================================================================================== */
#define MT_N 624
#define MT_M 397

typedef struct {
    uint32_t mt[MT_N];
    int index;
    int has_gauss_next;
    double gauss_next;
    uint64_t draws; /* number of random() calls (instrumentation) */
} pyrand;

/* init_genrand(s) */
static void pr_init_genrand(pyrand *r, uint32_t s) {
    r->mt[0] = s;
    for (int i = 1; i < MT_N; i++)
        r->mt[i] = 1812433253u * (r->mt[i - 1] ^ (r->mt[i - 1] >> 30)) + (uint32_t)i;
    r->index = MT_N;
}

/* init_by_array(key, key_length) */
static void pr_init_by_array(pyrand *r, const uint32_t *key, size_t klen) {
    pr_init_genrand(r, 19650218u);
    size_t i = 1, j = 0, k = (MT_N > klen ? MT_N : klen);
    uint32_t *mt = r->mt;
    for (; k; k--) {
        mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1664525u)) + key[j] + (uint32_t)j;
        i++;
        j++;
        if (i >= MT_N) {
            mt[0] = mt[MT_N - 1];
            i = 1;
        }
        if (j >= klen) j = 0;
    }
    for (k = MT_N - 1; k; k--) {
        mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1566083941u)) - (uint32_t)i;
        i++;
        if (i >= MT_N) {
            mt[0] = mt[MT_N - 1];
            i = 1;
        }
    }
    mt[0] = 0x80000000u;
}

/* random.seed(int): abs(int) as little-endian 32-bit words (at least one word), then
 * init_by_array; Random.seed also clears gauss_next. Seeds here are non-negative u64. */
static void pr_seed(pyrand *r, uint64_t s) {
    uint32_t key[2];
    size_t klen;
    key[0] = (uint32_t)s;
    key[1] = (uint32_t)(s >> 32);
    klen = key[1] ? 2 : 1;
    pr_init_by_array(r, key, klen);
    r->has_gauss_next = 0;
    r->gauss_next = 0.0;
    r->draws = 0;
}

/* genrand_uint32 */
static uint32_t pr_u32(pyrand *r) {
    static const uint32_t mag01[2] = {0x0u, 0x9908b0dfu};
    uint32_t y;
    uint32_t *mt = r->mt;
    if (r->index >= MT_N) {
        int kk;
        for (kk = 0; kk < MT_N - MT_M; kk++) {
            y = (mt[kk] & 0x80000000u) | (mt[kk + 1] & 0x7fffffffu);
            mt[kk] = mt[kk + MT_M] ^ (y >> 1) ^ mag01[y & 1u];
        }
        for (; kk < MT_N - 1; kk++) {
            y = (mt[kk] & 0x80000000u) | (mt[kk + 1] & 0x7fffffffu);
            mt[kk] = mt[kk + (MT_M - MT_N)] ^ (y >> 1) ^ mag01[y & 1u];
        }
        y = (mt[MT_N - 1] & 0x80000000u) | (mt[0] & 0x7fffffffu);
        mt[MT_N - 1] = mt[MT_M - 1] ^ (y >> 1) ^ mag01[y & 1u];
        r->index = 0;
    }
    y = mt[r->index++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}

/* random_random: 53-bit resolution */
static double pr_random(pyrand *r) {
    uint32_t a = pr_u32(r) >> 5, b = pr_u32(r) >> 6;
    r->draws++;
    return (a * 67108864.0 + b) * (1.0 / 9007199254740992.0);
}

/* Random.uniform: a + (b-a) * random() */
static double pr_uniform(pyrand *r, double a, double b) { return a + (b - a) * pr_random(r); }

/* Random.gauss (Lib/random.py, 3.10): pairwise cache */
static double pr_gauss(pyrand *r, double mu, double sigma) {
    double z;
    if (r->has_gauss_next) {
        z = r->gauss_next;
        r->has_gauss_next = 0;
    } else {
        const double TWOPI = 2.0 * 3.141592653589793;
        double x2pi = pr_random(r) * TWOPI;
        double g2rad = sqrt(-2.0 * log(1.0 - pr_random(r)));
        z = cos(x2pi) * g2rad;
        r->gauss_next = sin(x2pi) * g2rad;
        r->has_gauss_next = 1;
    }
    return mu + z * sigma;
}

void tgo_rng_words(uint64_t seed, int n, uint32_t *out) {
    pyrand r;
    pr_seed(&r, seed);
    for (int i = 0; i < n; i++) out[i] = pr_u32(&r);
}
void tgo_rng_random(uint64_t seed, int n, double *out) {
    pyrand r;
    pr_seed(&r, seed);
    for (int i = 0; i < n; i++) out[i] = pr_random(&r);
}
void tgo_rng_uniform5(uint64_t seed, double *out) {
    pyrand r;
    pr_seed(&r, seed);
    out[0] = pr_uniform(&r, 0.85, 1.0);
    out[1] = pr_uniform(&r, 0, 0.15);
    out[2] = pr_uniform(&r, 0, 1);
    out[3] = pr_uniform(&r, -4, -2.0);
    out[4] = pr_uniform(&r, 2.0, 4);
}
void tgo_rng_gauss(uint64_t seed, int pairs, double *out) {
    pyrand r;
    pr_seed(&r, seed);
    for (int i = 0; i < pairs; i++) {
        out[2 * i] = pr_gauss(&r, 0, 48 / 24.0);
        out[2 * i + 1] = pr_gauss(&r, 0, 48 / 36.0);
    }
}

/* ======================================================================================
 * Constants (_scale.py:8-9, _cell_types.py:7-13, _actions.py:7-13, IM/:15-16)
 * ====================================================================================== */
#define XSCALE 48
#define YSCALE 48
#define C_OPEN ' '
#define C_WALL '/'
#define C_LADDER 'L'
#define C_DOOR 'D'
enum { A_NOP = 0, A_UP, A_DOWN, A_LEFT, A_RIGHT, A_JUMP, A_INTERACT };
#define JUMP_REWARD (-5)
#define STEP_REWARD (-1)

#define MAXW 64
#define MAXH 64
#define MAXOBJ 32
#define MAXTRIG 16
#define MAXBAG 32

enum { O_DOOR, O_HANDLE, O_BOLT, O_KEY, O_GOLD };

typedef struct { /* one object line of domain-objects.txt */
    int type, cx, cy, flag;
} obj_spec;

typedef struct { /* one line of domain-interactions.txt */
    int type1, idx1, bool1, type2, idx2, bool2;
} trig_spec;

struct tgo_level {
    int W, H;
    char desc[MAXH][MAXW]; /* get_file_description (IM/:180-202) */
    int nobj;
    obj_spec objs[MAXOBJ];
    int ntrig;
    trig_spec trigs[MAXOBJ * 4];
};

/* ======================================================================================
 * Level parsing (IM/:75-202)
 * ====================================================================================== */
static int is_space(char c) { return c == ' ' || c == '\t' || c == '\r' || c == '\n' || c == '\f' || c == '\v'; }

static int split_words(char *line, char **w, int maxw) {
    int n = 0;
    char *p = line;
    while (*p) {
        while (*p && is_space(*p)) p++;
        if (!*p) break;
        if (n < maxw) w[n] = p;
        n++;
        while (*p && !is_space(*p)) p++;
        if (*p) *p++ = 0;
    }
    return n;
}

static int type_of(const char *s) {
    if (!strcmp(s, "door")) return O_DOOR;
    if (!strcmp(s, "handle")) return O_HANDLE;
    if (!strcmp(s, "bolt")) return O_BOLT;
    return -1;
}

tgo_level *tgo_level_parse(const char *domain, const char *objects, const char *interactions) {
    tgo_level *lv = (tgo_level *)calloc(1, sizeof(tgo_level));
    if (!lv) return NULL;
    /* description: each line str.strip()-ed (IM/:186-192) */
    const char *p = domain;
    int h = 0;
    while (*p) {
        const char *e = p;
        while (*e && *e != '\n') e++;
        const char *a = p, *b = e;
        while (a < b && is_space(*a)) a++;
        while (b > a && is_space(b[-1])) b--;
        if (h >= MAXH || b - a > MAXW) goto fail;
        /* readlines() yields every line incl. empty ones; the reference would then hold an
         * empty row. Our level files have none; reject such rows to stay in the spec. */
        if (b - a == 0) {
            if (*e == 0) break;
            goto fail;
        }
        for (int x = 0; x < b - a; x++) lv->desc[h][x] = a[x];
        if (h == 0) lv->W = (int)(b - a);
        else if (b - a != lv->W) goto fail;
        h++;
        p = *e ? e + 1 : e;
    }
    lv->H = h;
    if (lv->H == 0 || lv->W == 0) goto fail;

    /* read_objects (IM/:119-166): line.startswith(...) then split */
    {
        char buf[4096];
        size_t L = strlen(objects);
        if (L >= sizeof buf) goto fail;
        memcpy(buf, objects, L + 1);
        char *save = buf;
        while (save && *save) {
            char *nl = strchr(save, '\n');
            if (nl) *nl = 0;
            char *line = save;
            save = nl ? nl + 1 : NULL;
            char *w[8];
            int t = -1;
            if (!strncmp(line, "door", 4)) t = O_DOOR;
            else if (!strncmp(line, "key", 3)) t = O_KEY;
            else if (!strncmp(line, "bolt", 4)) t = O_BOLT;
            else if (!strncmp(line, "gold", 4)) t = O_GOLD;
            else if (!strncmp(line, "handle", 6)) t = O_HANDLE;
            if (t < 0) continue;
            int nw = split_words(line, w, 8);
            if (nw < 3 || lv->nobj >= MAXOBJ) goto fail;
            obj_spec *o = &lv->objs[lv->nobj++];
            o->type = t;
            o->cx = atoi(w[1]);
            o->cy = atoi(w[2]);
            o->flag = (t == O_DOOR || t == O_BOLT || t == O_HANDLE) ? (nw > 3 && !strcmp(w[3], "True")) : 0;
        }
    }
    /* extract_interactives (IM/:75-117) */
    {
        char buf[8192];
        size_t L = strlen(interactions);
        if (L >= sizeof buf) goto fail;
        memcpy(buf, interactions, L + 1);
        char *save = buf;
        while (save && *save) {
            char *nl = strchr(save, '\n');
            if (nl) *nl = 0;
            char *line = save;
            save = nl ? nl + 1 : NULL;
            char *w[8];
            int nw = split_words(line, w, 8);
            if (nw == 0) continue;
            if (nw != 6 || lv->ntrig >= MAXOBJ * 4) goto fail;
            trig_spec *t = &lv->trigs[lv->ntrig++];
            t->type1 = type_of(w[0]);
            t->idx1 = atoi(w[1]);
            t->bool1 = !strcmp(w[2], "True");
            t->type2 = type_of(w[3]);
            t->idx2 = atoi(w[4]);
            t->bool2 = !strcmp(w[5], "True");
            if (t->type1 < 0 || t->type2 < 0) goto fail;
        }
    }
    return lv;
fail:
    free(lv);
    return NULL;
}

void tgo_level_free(tgo_level *lv) { free(lv); }

/* ======================================================================================
 * Env (IM/:19-481 + OB/)
 * ====================================================================================== */
typedef struct {
    int type;
    int cx, cy, x, y; /* _GameObject (OB/:18-32) */
    double radius;
    int closed;       /* door */
    int up;           /* handle */
    int locked;       /* bolt */
    double angle;     /* handle */
    int prev;         /* previously_triggered */
    int nt, nf;
    int tt[MAXTRIG], ttv[MAXTRIG]; /* trigger_true (object indices) + vals */
    int tf[MAXTRIG], tfv[MAXTRIG];
} gobj;

struct tgo_env {
    const tgo_level *lv;
    pyrand rng;
    int W, H, width, height;
    char map[MAXH][MAXW]; /* the pixel map at cell granularity (see header comment) */
    int nobj;
    gobj obj[MAXOBJ];
    int doors[MAXOBJ], nd, handles[MAXOBJ], nh, bolts[MAXOBJ], nb;
    int bag[MAXBAG], nbag;
    int playerx, playery;
    int x_incr, y_incr, jump_ticker, player_width, player_height, facing_right;
    int64_t total_actions;
    int64_t ticks_total;
    int err;
};

static int pyfloordiv(int a, int b) { /* Python // for b > 0 */
    int q = a / b;
    if ((a % b) != 0 && (a < 0)) q--;
    return q;
}

/* door.update_map (OB/:246-253) */
static void door_update_map(tgo_env *e, gobj *d) {
    if (d->cy >= 0 && d->cy < e->H && d->cx >= 0 && d->cx < e->W)
        e->map[d->cy][d->cx] = d->closed ? C_DOOR : C_OPEN;
}

static void handle_wiggle(tgo_env *e, gobj *h) { /* set_angle_wiggle (OB/:127-131) */
    if (h->up) h->angle = pr_uniform(&e->rng, 0.85, 1.0);
    else h->angle = pr_uniform(&e->rng, 0, 0.15);
}

static void process_trigger(tgo_env *e, int oi, int val);

/* set_val per class: door OB/:231-235, handle OB/:145-149, bolt OB/:175-178, base OB/:73-74 */
static void set_val(tgo_env *e, int oi, int val) {
    gobj *o = &e->obj[oi];
    switch (o->type) {
    case O_DOOR:
        if (o->closed != val) {
            o->closed = val;
            door_update_map(e, o);
            process_trigger(e, oi, val);
        }
        break;
    case O_HANDLE:
        if (o->up != val) {
            o->up = val;
            handle_wiggle(e, o);
            process_trigger(e, oi, val);
        }
        break;
    case O_BOLT:
        if (o->locked != val) {
            o->locked = val;
            process_trigger(e, oi, val);
        }
        break;
    default:
        break;
    }
}

/* _GameObject.process_trigger (OB/:76-94) */
static void process_trigger(tgo_env *e, int oi, int val) {
    gobj *o = &e->obj[oi];
    o->prev = 1;
    if (val) {
        for (int i = 0; i < o->nt; i++)
            if (!e->obj[o->tt[i]].prev) set_val(e, o->tt[i], o->ttv[i]);
    } else {
        for (int i = 0; i < o->nf; i++)
            if (!e->obj[o->tf[i]].prev) set_val(e, o->tf[i], o->tfv[i]);
    }
    o->prev = 0;
}

/* handle.flip (OB/:117-122) */
static void handle_flip(tgo_env *e, int oi) {
    gobj *h = &e->obj[oi];
    if (pr_uniform(&e->rng, 0, 1) <= 0.8) set_val(e, oi, !h->up);
    else handle_wiggle(e, h);
}

/* near_enough (OB/:46-53) */
static int near_enough(const gobj *o, double x, double y) {
    double centerx = o->x + (XSCALE / 2.0);
    double centery = o->y + (YSCALE / 2.0);
    double dist = pow(x - centerx, 2) + pow(y - centery, 2);
    return sqrt(dist) < o->radius;
}

static void move_to(gobj *o, int cx, int cy) { /* OB/:34-38 */
    o->cx = cx;
    o->cy = cy;
    o->x = cx * XSCALE;
    o->y = cy * YSCALE;
}

/* build_map + read_objects + extract_interactives + player_initial_position
 * (IM/:55-73 reset_game, identical to the constructor IM/:31-53) */
static void reset_game(tgo_env *e) {
    const tgo_level *lv = e->lv;
    e->W = lv->W;
    e->H = lv->H;
    e->width = e->W * XSCALE;
    e->height = e->H * YSCALE;
    for (int y = 0; y < e->H; y++)
        for (int x = 0; x < e->W; x++) e->map[y][x] = lv->desc[y][x];
    /* read_objects (IM/:119-166) */
    e->nobj = lv->nobj;
    for (int i = 0; i < lv->nobj; i++) {
        const obj_spec *s = &lv->objs[i];
        gobj *o = &e->obj[i];
        memset(o, 0, sizeof *o);
        o->type = s->type;
        o->cx = s->cx;
        o->cy = s->cy;
        o->x = s->cx * XSCALE;
        o->y = s->cy * YSCALE;
        o->radius = XSCALE / 2.0;
        if (s->type == O_DOOR) {
            o->closed = s->flag;
            door_update_map(e, o); /* OB/:226 */
        } else if (s->type == O_BOLT) {
            o->locked = s->flag;
        } else if (s->type == O_HANDLE) {
            o->up = s->flag;
            if (o->up) o->angle = pr_uniform(&e->rng, 0.85, 1.0); /* OB/:111-114 */
            else o->angle = pr_uniform(&e->rng, 0, 0.15);
            o->radius = XSCALE * 0.75; /* OB/:115 */
        }
    }
    /* extract_interactives (IM/:75-117) */
    e->nd = e->nh = e->nb = 0;
    for (int i = 0; i < e->nobj; i++) {
        if (e->obj[i].type == O_DOOR) e->doors[e->nd++] = i;
        else if (e->obj[i].type == O_HANDLE) e->handles[e->nh++] = i;
        else if (e->obj[i].type == O_BOLT) e->bolts[e->nb++] = i;
    }
    for (int t = 0; t < lv->ntrig; t++) {
        const trig_spec *s = &lv->trigs[t];
        const int *l1 = s->type1 == O_HANDLE ? e->handles : s->type1 == O_BOLT ? e->bolts : e->doors;
        const int *l2 = s->type2 == O_DOOR ? e->doors : s->type2 == O_HANDLE ? e->handles : e->bolts;
        gobj *o = &e->obj[l1[s->idx1]];
        if (s->bool1) {
            o->tt[o->nt] = l2[s->idx2];
            o->ttv[o->nt++] = s->bool2;
        } else {
            o->tf[o->nf] = l2[s->idx2];
            o->tfv[o->nf++] = s->bool2;
        }
    }
    /* player_initial_position (IM/:168-178) */
    int nx = (int)pr_gauss(&e->rng, 0, XSCALE / 24.0);
    int ny = (int)fabs(pr_gauss(&e->rng, 0, YSCALE / 36.0));
    e->playerx = 0;
    e->playery = 0;
    int found = 0;
    for (int y = 0; y < e->H && !found; y++)
        for (int x = 0; x < e->W; x++)
            if (lv->desc[y][x] != C_WALL) {
                e->playerx = x * XSCALE + XSCALE / 2 + nx;
                e->playery = y * YSCALE + ny;
                found = 1;
                break;
            }
    e->nbag = 0;
    e->x_incr = XSCALE / 10;
    e->y_incr = YSCALE / 10;
    e->jump_ticker = 0;
    e->player_width = XSCALE / 2;
    e->player_height = YSCALE;
    e->facing_right = 1;
    e->total_actions = 0;
}

/* ---- map probes (IM/:218-230) -------------------------------------------------------- */
static char object_type_at(const tgo_env *e, int x, int y) {
    if (x >= e->width || x < 0) return C_WALL;
    if (y >= e->height || y < 0) return C_WALL;
    return e->map[y / YSCALE][x / XSCALE];
}
static char object_type_at_cell(const tgo_env *e, int xc, int yc) {
    return object_type_at(e, xc * XSCALE + XSCALE / 2, yc * YSCALE + YSCALE / 2);
}

/* ---- the six collision predicates, pixel loops as in the reference ------------------- */
static int up_clear(const tgo_env *e) { /* IM/:232-238 */
    int xo[3] = {-e->x_incr, 0, e->x_incr};
    for (int i = 0; i < 3; i++)
        for (int yoff = -e->y_incr; yoff < 0; yoff++)
            if (object_type_at(e, e->playerx + xo[i], e->playery + yoff) != C_OPEN) return 0;
    return 1;
}
static int can_go_up(const tgo_env *e) { /* IM/:240-250 */
    if (e->playery <= 1) return 0;
    int yo[3] = {-e->y_incr, 0, YSCALE - e->y_incr};
    int xo[2] = {pyfloordiv(-e->player_width, 2), e->player_width / 2};
    for (int j = 0; j < 3; j++)
        for (int i = 0; i < 2; i++)
            if (object_type_at(e, e->playerx + xo[i], e->playery + yo[j]) == C_LADDER) return 1;
    return 0;
}
static int can_go_down(const tgo_env *e) { /* IM/:252-257 */
    int xo[2] = {pyfloordiv(-e->player_width, 2), e->player_width / 2};
    for (int yoff = 0; yoff < YSCALE + e->y_incr; yoff++)
        for (int i = 0; i < 2; i++)
            if (object_type_at(e, e->playerx + xo[i], e->playery + yoff) == C_LADDER) return 1;
    return 0;
}
static int can_go_left(const tgo_env *e) { /* IM/:259-269 */
    int yo[2] = {e->y_incr, YSCALE - e->y_incr};
    int x = e->playerx - (e->player_width / 2) - e->x_incr;
    for (int j = 0; j < 2; j++) {
        if (object_type_at(e, x, e->playery + yo[j]) == C_WALL) return 0;
        if (object_type_at(e, x, e->playery + yo[j]) == C_DOOR) return 0;
    }
    return 1;
}
static int can_go_right(const tgo_env *e) { /* IM/:271-281 */
    int yo[2] = {e->y_incr, YSCALE - e->y_incr};
    int x = e->playerx + (e->player_width / 2) + e->x_incr;
    for (int j = 0; j < 2; j++) {
        if (object_type_at(e, x, e->playery + yo[j]) == C_WALL) return 0;
        if (object_type_at(e, x, e->playery + yo[j]) == C_DOOR) return 0;
    }
    return 1;
}
static int can_fall(const tgo_env *e) { /* IM/:283-288 */
    int xo[2] = {pyfloordiv(-e->player_width, 2) + 2, -2 + e->player_width / 2};
    int yo[2] = {0, YSCALE + 2};
    for (int i = 0; i < 2; i++)
        for (int j = 0; j < 2; j++)
            if (object_type_at(e, e->playerx + xo[i], e->playery + yo[j]) != C_OPEN) return 0;
    return 1;
}

/* ---- bag helpers (IM/:402-445) --------------------------------------------------------- */
static int is_object_at(const tgo_env *e, int xc, int yc) {
    for (int i = 0; i < e->nobj; i++) {
        const gobj *o = &e->obj[i];
        if (o->cx == xc && o->cy == yc) {
            if (o->type == O_HANDLE || (o->type == O_DOOR && o->closed) || o->type == O_BOLT ||
                o->type == O_GOLD || o->type == O_KEY)
                return 1;
        }
    }
    return 0;
}
static int is_closed_door_at(const tgo_env *e, int xc, int yc) {
    for (int i = 0; i < e->nobj; i++) {
        const gobj *o = &e->obj[i];
        if (o->cx == xc && o->cy == yc && o->type == O_DOOR && o->closed) return 1;
    }
    return 0;
}
static int player_got_key(const tgo_env *e) {
    for (int i = 0; i < e->nbag; i++)
        if (e->obj[e->bag[i]].type == O_KEY) return 1;
    return 0;
}
static int player_got_goldcoin(const tgo_env *e) {
    for (int i = 0; i < e->nbag; i++)
        if (e->obj[e->bag[i]].type == O_GOLD) return 1;
    return 0;
}
static void drop_key(tgo_env *e) {
    for (int i = 0; i < e->nbag; i++)
        if (e->obj[e->bag[i]].type == O_KEY) {
            int oi = e->bag[i];
            memmove(&e->bag[i], &e->bag[i + 1], (size_t)(e->nbag - i - 1) * sizeof(int));
            e->nbag--;
            move_to(&e->obj[oi], -1, -1);
            return;
        }
}
static void get_player_cell(const tgo_env *e, int *xc, int *yc) {
    *xc = pyfloordiv(e->playerx, XSCALE);
    *yc = pyfloordiv(e->playery + (YSCALE / 2), YSCALE);
}

/* noisy (IM/:361-366): round() is half-to-even == rint() in the default rounding mode */
static int noisy(tgo_env *e, int val) {
    double between = val / 2.0;
    if (val < between) return (int)rint(pr_uniform(&e->rng, val, between));
    return (int)rint(pr_uniform(&e->rng, between, val));
}

/* _TreasureGameImpl.step (IM/:290-359) */
static int prim_step(tgo_env *e, int action) {
    int xdelta = 0, ydelta = 0;
    e->total_actions++;
    e->ticks_total++;
    if (action == A_UP) {
        if (can_go_up(e)) ydelta = noisy(e, -e->y_incr);
    } else if (action == A_DOWN) {
        if (can_go_down(e)) ydelta = noisy(e, e->y_incr);
    } else if (action == A_LEFT) {
        if (can_go_left(e)) {
            xdelta = noisy(e, -e->x_incr);
            e->facing_right = 0;
        }
    } else if (action == A_RIGHT) {
        if (can_go_right(e)) {
            xdelta = noisy(e, e->x_incr);
            e->facing_right = 1;
        }
    } else if (action == A_JUMP) {
        if (!can_go_down(e) && up_clear(e)) {
            e->jump_ticker = 22;
            if (pr_random(&e->rng) > 0.25) e->jump_ticker = 23;
        }
    } else if (action == A_INTERACT) {
        for (int i = 0; i < e->nobj; i++) {
            gobj *o = &e->obj[i];
            if (near_enough(o, e->playerx, e->playery + YSCALE / 2.0)) {
                if (o->type == O_HANDLE) handle_flip(e, i);
                else if (o->type == O_BOLT) {
                    if (player_got_key(e)) {
                        set_val(e, i, 0); /* try_unlock -> bolt.unlock (IM/:430-432, OB/:172) */
                        drop_key(e);
                    }
                }
            }
        }
    }
    if (e->jump_ticker > 0) {
        if (up_clear(e)) ydelta = -e->y_incr;
        e->jump_ticker = e->jump_ticker - 1;
    } else if (can_fall(e)) {
        e->jump_ticker = 0;
        ydelta = e->y_incr;
    }
    e->playerx = e->playerx + xdelta;
    if (can_fall(e) && ydelta > 0) {
        while (ydelta > 0) {
            e->playery = e->playery + 1;
            ydelta = ydelta - 1;
            if (!can_fall(e)) ydelta = 0;
        }
    } else {
        e->playery = e->playery + ydelta;
    }
    for (int i = 0; i < e->nobj; i++) {
        gobj *o = &e->obj[i];
        if (o->type == O_KEY || o->type == O_GOLD) {
            if (near_enough(o, e->playerx, e->playery + YSCALE / 2.0)) {
                move_to(o, e->W - 1 - e->nbag, e->H - 1);
                if (e->nbag < MAXBAG) e->bag[e->nbag++] = i;
                else e->err = 1;
            }
        }
    }
    return action == A_JUMP ? JUMP_REWARD : STEP_REWARD;
}

/* get_state (IM/:368-378) with the per-object get_state of OB/ */
static void get_state(const tgo_env *e, double obs[9]) {
    int k = 0;
    obs[k++] = (double)e->playerx / e->width;
    obs[k++] = (double)e->playery / e->height;
    for (int i = 0; i < e->nobj && k < 9; i++) {
        const gobj *o = &e->obj[i];
        double ww = e->W * XSCALE, wh = e->H * YSCALE; /* world_width/height (OB/:25-26) */
        if (o->type == O_HANDLE) obs[k++] = o->angle;
        else if (o->type == O_BOLT) obs[k++] = o->locked ? 1.0 : 0.0;
        else if (o->type == O_GOLD || o->type == O_KEY) {
            obs[k++] = (double)o->x / ww;
            if (k < 9) obs[k++] = (double)o->y / wh;
        }
    }
}

/* ======================================================================================
 * Options (MO/) — one run() of option k (OP/:20-36)
 * ====================================================================================== */
enum { OPT_GO_LEFT, OPT_GO_RIGHT, OPT_UP_LADDER, OPT_DOWN_LADDER, OPT_INTERACT, OPT_DOWN_LEFT,
       OPT_DOWN_RIGHT, OPT_JUMP_LEFT, OPT_JUMP_RIGHT }; /* create_options order, IM/:495 */

/* go_left/go_right is_target_cell (MO/:54-67, MO/:126-139); dir = -1 / +1 */
static int go_is_target_cell(const tgo_env *e, int dir, int xc, int yc) {
    if (object_type_at_cell(e, xc, yc - 1) == C_LADDER) return 1;
    if (object_type_at_cell(e, xc, yc + 1) == C_LADDER) return 1;
    if (object_type_at_cell(e, xc + dir, yc) == C_WALL) return 1;
    if (is_object_at(e, xc, yc) || is_closed_door_at(e, xc + dir, yc)) return 1;
    if (object_type_at_cell(e, xc + dir, yc + 1) == C_OPEN) return 1;
    return 0;
}
/* get_target_cell (MO/:43-52 left, MO/:115-124 right; the right one's xc<0 test is dead) */
static int go_get_target_cell(const tgo_env *e, int dir, int pxc, int pyc, int *txc) {
    int xc = pxc + dir, yc = pyc;
    while (!go_is_target_cell(e, dir, xc, yc)) {
        xc = xc + dir;
        if (xc < 0) return 0;
    }
    *txc = xc;
    return 1;
}
/* can_run (MO/:23-41, MO/:95-113) */
static int go_can_run(const tgo_env *e, int dir) {
    int xc, yc, tc;
    get_player_cell(e, &xc, &yc);
    if (!go_get_target_cell(e, dir, xc, yc, &tc)) return 0;
    while (dir < 0 ? xc >= tc : xc <= tc) {
        if (object_type_at_cell(e, xc, yc) != C_OPEN) return 0;
        if (object_type_at_cell(e, xc, yc + 1) == C_OPEN) return 0;
        xc += dir;
    }
    return 1;
}
static int close_enough_x(const tgo_env *e, int txc) { /* MO/:69-72 etc. */
    double tx = (txc * XSCALE) + (XSCALE / 2.0);
    double diff = fabs(tx - e->playerx);
    return diff < e->x_incr;
}
/* down_left / down_right can_run (MO/:199-209, MO/:394-404) */
static int down_can_run(const tgo_env *e, int dir) {
    int xc, yc;
    get_player_cell(e, &xc, &yc);
    if (object_type_at_cell(e, xc + dir, yc) != C_OPEN) return 0;
    if (object_type_at_cell(e, xc + dir, yc + 1) != C_OPEN) return 0;
    return 1;
}
static int down_get_target_cell(const tgo_env *e, int dir, int pxc, int pyc, int *txc) {
    int xc = pxc + dir, yc = pyc + 1; /* MO/:211-221, MO/:406-416 */
    while (object_type_at_cell(e, xc, yc) == C_OPEN) {
        yc = yc + 1;
        if (yc >= e->H) return 0;
    }
    *txc = xc;
    return 1;
}
static int landing(const tgo_env *e, int xc, int yc) { /* MO/:281-287, MO/:351-357 */
    if (object_type_at_cell(e, xc, yc) != C_OPEN) return 0;
    if (object_type_at_cell(e, xc, yc + 1) != C_WALL) return 0;
    return 1;
}
static int jump_can_run(const tgo_env *e, int dir) { /* MO/:254-267, MO/:324-337 */
    int xc, yc;
    get_player_cell(e, &xc, &yc);
    if (object_type_at_cell(e, xc, yc - 1) != C_OPEN) return 0;
    if (object_type_at_cell(e, xc + dir, yc - 1) != C_OPEN) return 0;
    if (!(landing(e, xc + dir, yc - 1) || landing(e, xc + 2 * dir, yc - 1))) return 0;
    return 1;
}
static int jump_get_target_cell(const tgo_env *e, int dir, int pxc, int pyc, int *txc) {
    if (landing(e, pxc + dir, pyc - 1)) { /* MO/:269-279, MO/:339-349 */
        *txc = pxc + dir;
        return 1;
    } else if (landing(e, pxc + 2 * dir, pyc - 1)) {
        *txc = pxc + 2 * dir;
        return 1;
    }
    return 0;
}
static int interact_can_run(const tgo_env *e) { /* MO/:446-455 */
    for (int i = 0; i < e->nobj; i++) {
        const gobj *o = &e->obj[i];
        if (near_enough(o, e->playerx, e->playery + YSCALE / 2.0)) {
            if (o->type == O_HANDLE) return 1;
            else if (o->type == O_BOLT) {
                if (player_got_key(e)) return 1;
            }
        }
    }
    return 0;
}

static int option_can_run(const tgo_env *e, int k) {
    switch (k) {
    case OPT_GO_LEFT: return go_can_run(e, -1);
    case OPT_GO_RIGHT: return go_can_run(e, +1);
    case OPT_UP_LADDER: return can_go_up(e);   /* MO/:165-166 */
    case OPT_DOWN_LADDER: return can_go_down(e); /* MO/:181-182 */
    case OPT_INTERACT: return interact_can_run(e);
    case OPT_DOWN_LEFT: return down_can_run(e, -1);
    case OPT_DOWN_RIGHT: return down_can_run(e, +1);
    case OPT_JUMP_LEFT: return jump_can_run(e, -1);
    case OPT_JUMP_RIGHT: return jump_can_run(e, +1);
    }
    return 0;
}

/* option-local state: start_cell/target_cell (None between runs) + done */
typedef struct {
    int have_cells, txc, done;
} optstate;

/* policy_step of every option (MO/) */
static int policy_step(tgo_env *e, int k, optstate *s) {
    int xc, yc;
    switch (k) {
    case OPT_GO_LEFT:
    case OPT_GO_RIGHT: { /* MO/:74-85, MO/:146-157 */
        int dir = k == OPT_GO_LEFT ? -1 : 1;
        if (!s->have_cells) {
            get_player_cell(e, &xc, &yc);
            if (!go_get_target_cell(e, dir, xc, yc, &s->txc)) e->err = 2;
            s->have_cells = 1;
        }
        if (close_enough_x(e, s->txc)) {
            s->done = 1;
            s->have_cells = 0;
        }
        return dir < 0 ? A_LEFT : A_RIGHT;
    }
    case OPT_UP_LADDER: /* MO/:168-173 */
        if (!can_go_up(e)) {
            s->done = 1;
            return A_NOP;
        }
        return A_UP;
    case OPT_DOWN_LADDER: /* MO/:184-189 */
        if (!can_go_down(e)) {
            s->done = 1;
            return A_NOP;
        }
        return A_DOWN;
    case OPT_INTERACT: /* MO/:457-460 */
        s->done = 1;
        return A_INTERACT;
    case OPT_DOWN_LEFT:
    case OPT_DOWN_RIGHT: { /* MO/:231-244, MO/:426-439 */
        int dir = k == OPT_DOWN_LEFT ? -1 : 1;
        if (!s->have_cells) {
            get_player_cell(e, &xc, &yc);
            if (!down_get_target_cell(e, dir, xc, yc, &s->txc)) e->err = 2;
            s->have_cells = 1;
        }
        if (close_enough_x(e, s->txc)) {
            if (!can_fall(e)) {
                s->done = 1;
                s->have_cells = 0;
            }
            return A_NOP;
        }
        return dir < 0 ? A_LEFT : A_RIGHT;
    }
    case OPT_JUMP_LEFT:
    case OPT_JUMP_RIGHT: { /* MO/:297-314, MO/:367-384 */
        int dir = k == OPT_JUMP_LEFT ? -1 : 1;
        if (!s->have_cells) {
            get_player_cell(e, &xc, &yc);
            if (!jump_get_target_cell(e, dir, xc, yc, &s->txc)) e->err = 2;
            s->have_cells = 1;
            return A_JUMP;
        }
        if (close_enough_x(e, s->txc)) {
            if (!can_fall(e)) {
                s->done = 1;
                s->have_cells = 0;
            }
            return A_NOP;
        }
        if (dir < 0) return (!can_fall(e) && !can_go_left(e)) ? A_RIGHT : A_LEFT;
        return (!can_fall(e) && !can_go_right(e)) ? A_LEFT : A_RIGHT;
    }
    }
    return A_NOP;
}

/* _Option.run (OP/:20-36). Returns 1 and *rew if it ran, 0 if it could not run (None). */
static int option_run(tgo_env *e, int k, int *rew) {
    if (!option_can_run(e, k)) return 0;
    optstate s = {0, 0, 0};
    int tot = 0;
    while (!s.done) {
        int act = policy_step(e, k, &s);
        tot += prim_step(e, act);
        if (e->err) break;
    }
    *rew = tot;
    return 1;
}

/* ======================================================================================
 * Public single-env API (TG/:54-114)
 * ====================================================================================== */
size_t tgo_env_size(void) { return sizeof(tgo_env); }

static void env_init(tgo_env *e, const tgo_level *lv, uint64_t seed, double obs[9]) {
    memset(e, 0, sizeof *e);
    e->lv = lv;
    pr_seed(&e->rng, seed); /* random.seed(seed) */
    reset_game(e);          /* TreasureGame.__init__ -> _TreasureGameImpl.__init__ (TG/:69) */
    reset_game(e);          /* env.reset() (TG/:78-81) */
    e->ticks_total = 0;
    if (obs) get_state(e, obs);
}

tgo_env *tgo_env_new(const tgo_level *lv, uint64_t seed, double obs[9]) {
    tgo_env *e = (tgo_env *)malloc(sizeof(tgo_env));
    if (e) env_init(e, lv, seed, obs);
    return e;
}
void tgo_env_free(tgo_env *e) { free(e); }

/* TreasureGame.step (TG/:91-96) */
int tgo_step(tgo_env *e, int action, double obs[9], int32_t *reward, uint8_t *valid,
             uint8_t *done) {
    if (action < -9 || action > 8) return -1; /* option_list[action]: IndexError */
    if (action < 0) action += 9;
    int r = 0;
    int ran = option_run(e, action, &r);
    if (obs) get_state(e, obs);
    if (reward) *reward = ran ? r : 0;
    if (valid) *valid = (uint8_t)ran;
    int xc, yc;
    get_player_cell(e, &xc, &yc);
    if (done) *done = (uint8_t)(player_got_goldcoin(e) && yc == 0);
    return e->err ? -2 : 0;
}

void tgo_reset(tgo_env *e, double obs[9]) { /* TG/:78-81 */
    reset_game(e);
    if (obs) get_state(e, obs);
}

unsigned tgo_mask(tgo_env *e) { /* available_mask (TG/:83-89) */
    unsigned m = 0;
    for (int k = 0; k < 9; k++) m |= (unsigned)option_can_run(e, k) << k;
    return m;
}
uint64_t tgo_draws(const tgo_env *e) { return e->rng.draws; }
int64_t tgo_ticks(const tgo_env *e) { return e->ticks_total; }

void tgo_internal(const tgo_env *e, int32_t out[12]) {
    int doors = 0, handles = 0, bolt = 0, kx = 0, ky = 0, gx = 0, gy = 0;
    for (int i = 0; i < e->nd; i++) doors |= e->obj[e->doors[i]].closed << i;
    for (int i = 0; i < e->nh; i++) handles |= e->obj[e->handles[i]].up << i;
    if (e->nb) bolt = e->obj[e->bolts[0]].locked;
    for (int i = 0; i < e->nobj; i++) {
        if (e->obj[i].type == O_KEY) { kx = e->obj[i].cx; ky = e->obj[i].cy; }
        if (e->obj[i].type == O_GOLD) { gx = e->obj[i].cx; gy = e->obj[i].cy; }
    }
    int32_t v[12] = {e->playerx, e->playery, e->jump_ticker, doors, handles, bolt,
                     kx, ky, gx, gy, e->facing_right, (int32_t)e->total_actions};
    memcpy(out, v, sizeof v);
}

unsigned tgo_predicates(tgo_env *e, int px, int py, unsigned door_bits) {
    int spx = e->playerx, spy = e->playery;
    char saved[MAXH][MAXW];
    memcpy(saved, e->map, sizeof saved);
    for (int i = 0; i < e->nd; i++) {
        gobj *d = &e->obj[e->doors[i]];
        int c = (door_bits >> i) & 1;
        if (d->cy >= 0 && d->cy < e->H && d->cx >= 0 && d->cx < e->W)
            e->map[d->cy][d->cx] = c ? C_DOOR : C_OPEN;
    }
    e->playerx = px;
    e->playery = py;
    unsigned m = (unsigned)up_clear(e) | (unsigned)can_go_up(e) << 1 | (unsigned)can_go_down(e) << 2 |
                 (unsigned)can_go_left(e) << 3 | (unsigned)can_go_right(e) << 4 |
                 (unsigned)can_fall(e) << 5;
    e->playerx = spx;
    e->playery = spy;
    memcpy(e->map, saved, sizeof saved);
    return m;
}

void tgo_predicate_table(tgo_env *e, int x0, int x1, int y0, int y1, unsigned door_bits,
                         uint8_t *out) {
    for (int y = y0; y < y1; y++)
        for (int x = x0; x < x1; x++)
            out[(size_t)(y - y0) * (size_t)(x1 - x0) + (size_t)(x - x0)] =
                (uint8_t)tgo_predicates(e, x, y, door_bits);
}

/* ======================================================================================
 * Action stream + hash (same as tests/golden/make_golden.py)
 * ====================================================================================== */
uint64_t tgo_sm64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
uint64_t tgo_action_hash(uint64_t a0, uint64_t g, uint64_t t) {
    return tgo_sm64(tgo_sm64(a0 ^ tgo_sm64(g)) ^ t);
}
int tgo_pick_action(uint64_t a0, uint64_t g, uint64_t t, int masked, unsigned mask) {
    uint64_t h = tgo_action_hash(a0, g, t);
    if (!masked) return (int)(h % 9);
    int c = __builtin_popcount(mask & 0x1FFu);
    if (c == 0) return (int)(h % 9);
    uint64_t k = h % (uint64_t)c;
    for (int i = 0; i < 9; i++)
        if (mask >> i & 1u) {
            if (k == 0) return i;
            k--;
        }
    return 0;
}
uint64_t tgo_rec_hash(uint64_t h, const double obs[9], int32_t reward, int valid, int done) {
    for (int i = 0; i < 9; i++) {
        uint64_t b;
        memcpy(&b, &obs[i], 8);
        h = tgo_sm64(h ^ b);
    }
    uint64_t w = (uint64_t)(uint32_t)reward | ((uint64_t)(valid & 0xFF) << 32) |
                 ((uint64_t)(done & 0xFF) << 40);
    return tgo_sm64(h ^ w);
}

/* ======================================================================================
 * Batched driver
 * ====================================================================================== */
int tgo_run(const tgo_level *lv, uint64_t seed_base, int64_t g0, int64_t n, int steps,
            uint64_t action_seed, int policy, int autoreset, double *obs, int32_t *reward,
            uint8_t *valid, uint8_t *done, double *final_obs, uint64_t *hash, int64_t *draws,
            int64_t *ticks, int nthreads) {
    int err = 0;
    const int64_t T1 = (int64_t)steps + 1;
#ifdef _OPENMP
    if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 16) num_threads(nthreads) reduction(| : err)
#endif
    for (int64_t i = 0; i < n; i++) {
        uint64_t g = (uint64_t)(g0 + i);
        tgo_env *e = (tgo_env *)malloc(sizeof(tgo_env));
        if (!e) {
            err |= 1;
            continue;
        }
        double o[9], fo[9];
        env_init(e, lv, seed_base + g, o);
        uint64_t h = tgo_rec_hash(g, o, 0, 0, 0);
        if (obs) memcpy(&obs[(i * T1) * 9], o, sizeof o);
        if (final_obs) memcpy(&final_obs[(i * T1) * 9], o, sizeof o);
        if (reward) reward[i * T1] = 0;
        if (valid) valid[i * T1] = 0;
        if (done) done[i * T1] = 0;
        for (int t = 0; t < steps; t++) {
            unsigned m = policy ? tgo_mask(e) : 0;
            int a = tgo_pick_action(action_seed, g, (uint64_t)t, policy, m);
            int32_t r;
            uint8_t v, d;
            if (tgo_step(e, a, fo, &r, &v, &d)) err |= 1;
            memcpy(o, fo, sizeof o);
            if (autoreset && d) tgo_reset(e, o);
            h = tgo_rec_hash(h, fo, r, v, d);
            int64_t j = i * T1 + t + 1;
            if (obs) memcpy(&obs[j * 9], o, sizeof o);
            if (final_obs) memcpy(&final_obs[j * 9], fo, sizeof fo);
            if (reward) reward[j] = r;
            if (valid) valid[j] = v;
            if (done) done[j] = d;
        }
        if (hash) hash[i] = h;
        if (draws) draws[i] = (int64_t)e->rng.draws;
        if (ticks) ticks[i] = e->ticks_total;
        free(e);
    }
    return err ? -1 : 0;
}

/* Episodes of an auto-reset run (the step driver above, reset() after a step that returned
 * done, TG/:91-96 + TG/:78-81): the (env, return, length) record of every episode whose last
 * step has index >= t_from, reduced to a count and the order-independent digest of
 * gym-treasure-game_amd/dist.py episode_digest: the sum mod 2^64 of
 * sm64(sm64(env) ^ (return & 0xFFFFFFFF | length << 32)). */
int tgo_run_episodes(const tgo_level *lv, uint64_t seed_base, int64_t g0, int64_t n, int steps,
                     uint64_t action_seed, int policy, int t_from, int64_t *count,
                     uint64_t *digest, int nthreads) {
    int err = 0;
    int64_t cnt = 0;
    uint64_t dig = 0;
#ifdef _OPENMP
    if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 16) num_threads(nthreads) reduction(| : err) \
    reduction(+ : cnt, dig)
#endif
    for (int64_t i = 0; i < n; i++) {
        uint64_t g = (uint64_t)(g0 + i);
        tgo_env *e = (tgo_env *)malloc(sizeof(tgo_env));
        if (!e) {
            err |= 1;
            continue;
        }
        double o[9], fo[9];
        env_init(e, lv, seed_base + g, o);
        int64_t ret = 0, len = 0;
        for (int t = 0; t < steps; t++) {
            unsigned m = policy ? tgo_mask(e) : 0;
            int a = tgo_pick_action(action_seed, g, (uint64_t)t, policy, m);
            int32_t r;
            uint8_t v, d;
            if (tgo_step(e, a, fo, &r, &v, &d)) err |= 1;
            ret += r;
            len += 1;
            if (d) {
                if (t >= t_from) {
                    const uint64_t packed = ((uint64_t)ret & 0xFFFFFFFFull) | ((uint64_t)len << 32);
                    dig += tgo_sm64(tgo_sm64(g) ^ packed);
                    cnt += 1;
                }
                tgo_reset(e, o);
                ret = len = 0;
            }
        }
        free(e);
    }
    *count = cnt;
    *digest = dig;
    return err ? -1 : 0;
}

/* ======================================================================================
 * Renderer: TreasureGame.render('rgb_array') (TG/:98-105) -> _TreasureGameDrawer.draw_domain
 * (DR/ = _treasure_game_impl/_treasure_game_drawer.py, DR/:136-163, DR/:238-269).
 *
 * PARITY UNPINNED: pygame is absent from this image, so the reference renderer cannot run
 * here and no reference frame exists to check against.  This section restates pygame 1.9.6 /
 * SDL 1.2 (the versions the reference's Python 3.7 era pulls in) as documented in DESIGN.md:
 *   - transform.scale: transform.c stretch() (Bresenham step, source index floor(d*s/D));
 *   - blit of a convert_alpha() sprite onto the convert()ed screen: SDL_blit_A.c
 *     BlitRGBtoRGBPixelAlpha, i.e. per channel d + ((s - d) * a >> 8), a == 255 copies,
 *     a == 0 skips;
 *   - draw.line(width 5): draw.c clip_and_draw_line_width -> 5 one-pixel lines offset along
 *     x or y, each drawline() (Bresenham, both end points, error term starting at 0);
 *   - draw.circle(r, width 0): draw.c draw_fillellipse (SDL_gfx filled-ellipse scanlines);
 *   - random_generator.choice: CPython Random.choice = seq[_randbelow(len)] with
 *     getrandbits(bit_length(len)) rejection (pinned against Python's random in the tests).
 * The screen is XRGB8888; the frame is its RGB bytes, rows top to bottom
 * (surfarray.array3d(...).swapaxes(0, 1)).  Sprites come in as RGBA8 (PIL decode of the
 * reference's PNGs, or synthetic sheets in the tests) in TGO_SPR_* order.
 * ====================================================================================== */
enum { /* sprite sheet order (shared with include/tg_amd.h TG_SPR_*) */
    TGO_SPR_BACKGROUND = 0, /* 5 variants: sprites/background/background_{0..4}.png */
    TGO_SPR_WALL = 5,       /* 5 variants: sprites/wall/wall_{0..4}.png */
    TGO_SPR_FLOOR = 10,     /* 5 variants: sprites/floor/floor-{0..4}.png */
    TGO_SPR_LADDER = 15, TGO_SPR_DOOR_CLOSED, TGO_SPR_DOOR_OPEN, TGO_SPR_KEY, TGO_SPR_GOLD,
    TGO_SPR_BOLT_OPEN, TGO_SPR_BOLT_LOCKED, TGO_SPR_HERO, TGO_SPR_HANDLE_BASE, TGO_SPR_COUNT
};

typedef struct {
    int w, h;
    uint32_t *px; /* ARGB8888, row-major */
} surf;

/* pygame transform.c stretch(): nearest neighbour with a Bresenham error term */
static void stretch(const surf *src, surf *dst) {
    const int dw2 = dst->w << 1, dh2 = dst->h << 1, sw2 = src->w << 1, sh2 = src->h << 1;
    int h_err = sh2 - dh2;
    int srow = 0;
    for (int looph = 0; looph < dst->h; ++looph) {
        int w_err = sw2 - dw2, sx = 0;
        for (int loopw = 0; loopw < dst->w; ++loopw) {
            dst->px[looph * dst->w + loopw] = src->px[srow * src->w + sx];
            while (w_err >= 0) {
                ++sx;
                w_err -= dw2;
            }
            w_err += sw2;
        }
        while (h_err >= 0) {
            ++srow;
            h_err -= dh2;
        }
        h_err += sh2;
    }
}

/* SDL_blit_A.c BlitRGBtoRGBPixelAlpha for one pixel (dst alpha is not displayed) */
static uint32_t blend_px(uint32_t d, uint32_t s) {
    const uint32_t a = s >> 24;
    if (a == 0) return d;
    if (a == 255) return (s & 0x00ffffffu) | (d & 0xff000000u);
    uint32_t out = d & 0xff000000u;
    for (int sh = 0; sh < 24; sh += 8) {
        const int sc = (int)((s >> sh) & 0xff), dc = (int)((d >> sh) & 0xff);
        const int c = dc + (((sc - dc) * (int)a) >> 8); /* arithmetic shift == floor */
        out |= (uint32_t)(c & 0xff) << sh;
    }
    return out;
}

/* Surface.blit(src, (x, y)) with SDL's clipping to the destination */
static void blit(surf *dst, const surf *src, int x, int y, int flip_x) {
    for (int j = 0; j < src->h; ++j) {
        const int yy = y + j;
        if (yy < 0 || yy >= dst->h) continue;
        for (int i = 0; i < src->w; ++i) {
            const int xx = x + i;
            if (xx < 0 || xx >= dst->w) continue;
            const int si = flip_x ? src->w - 1 - i : i; /* transform.flip(img, True, False) */
            uint32_t *p = &dst->px[yy * dst->w + xx];
            *p = blend_px(*p, src->px[j * src->w + si]);
        }
    }
}

static void set_at(surf *s, int x, int y, uint32_t c) {
    if (x >= 0 && y >= 0 && x < s->w && y < s->h) s->px[y * s->w + x] = c;
}

/* draw.c drawline(): Bresenham over the longer axis, both end points drawn */
static void drawline(surf *s, uint32_t color, int x1, int y1, int x2, int y2) {
    int deltax = x2 - x1, deltay = y2 - y1;
    const int signx = deltax < 0 ? -1 : 1, signy = deltay < 0 ? -1 : 1;
    deltax = signx * deltax + 1;
    deltay = signy * deltay + 1;
    int px = signx, py = 0, qx = 0, qy = signy; /* major step (px,py), minor step (qx,qy) */
    if (deltax < deltay) {                      /* swap axis if rise > run */
        int t = deltax;
        deltax = deltay;
        deltay = t;
        px = 0, py = signy, qx = signx, qy = 0;
    }
    int x = x1, y = y1, err = 0;
    for (int k = 0; k < deltax; ++k) {
        set_at(s, x, y, color);
        err += deltay;
        x += px, y += py;
        if (err >= deltax) {
            err -= deltax;
            x += qx, y += qy;
        }
    }
}

/* draw.c clip_and_draw_line(): the renderer only draws lines that lie inside the surface
 * (tgo_render checks), so clipline() is the accept case; horizontal / vertical lines cover
 * the same pixels as drawline(). */
static int clip_and_draw_line(surf *s, uint32_t color, const int *p) {
    if (p[0] < 0 || p[2] < 0 || p[1] < 0 || p[3] < 0 || p[0] >= s->w || p[2] >= s->w ||
        p[1] >= s->h || p[3] >= s->h)
        return -1;
    drawline(s, color, p[0], p[1], p[2], p[3]);
    return 0;
}

/* draw.c clip_and_draw_line_width(): width-1 extra lines offset by +1, -1, +2, -2 along y
 * for a mostly-horizontal line, else along x */
static int clip_and_draw_line_width(surf *s, uint32_t color, int width, const int *pts) {
    int xinc = 0, yinc = 0, rc = 0, np[4];
    if (abs(pts[0] - pts[2]) > abs(pts[1] - pts[3])) yinc = 1;
    else xinc = 1;
    rc |= clip_and_draw_line(s, color, pts);
    for (int loop = 1; loop < width; loop += 2) {
        const int o = loop / 2 + 1;
        np[0] = pts[0] + xinc * o, np[1] = pts[1] + yinc * o;
        np[2] = pts[2] + xinc * o, np[3] = pts[3] + yinc * o;
        rc |= clip_and_draw_line(s, color, np);
        if (loop + 1 < width) {
            np[0] = pts[0] - xinc * o, np[1] = pts[1] - yinc * o;
            np[2] = pts[2] - xinc * o, np[3] = pts[3] - yinc * o;
            rc |= clip_and_draw_line(s, color, np);
        }
    }
    return rc;
}

static void hline(surf *s, uint32_t color, int x1, int y, int x2) {
    for (int x = x1; x <= x2; ++x) set_at(s, x, y, color);
}

/* draw.c draw_fillellipse(x, y, rx, ry) with rx == ry (SDL_gfx filledEllipse scanlines) */
static void fillellipse(surf *s, int x, int y, int rx, int ry, uint32_t color) {
    int ix, iy, h, i, j, k, oh, oi, oj, ok;
    if (rx == 0 && ry == 0) {
        set_at(s, x, y, color);
        return;
    }
    oh = oi = oj = ok = 0xFFFF;
    if (rx > ry) {
        ix = 0;
        iy = rx * 64;
        do {
            h = (ix + 16) >> 6;
            i = (iy + 16) >> 6;
            j = (h * ry) / rx;
            k = (i * ry) / rx;
            if ((ok != k) && (oj != k)) {
                if (k) {
                    hline(s, color, x - h, y - k, x + h);
                    hline(s, color, x - h, y + k, x + h);
                } else {
                    hline(s, color, x - h, y, x + h);
                }
                ok = k;
            }
            if ((oj != j) && (ok != j) && (k != j)) {
                if (j) {
                    hline(s, color, x - i, y - j, x + i);
                    hline(s, color, x - i, y + j, x + i);
                } else {
                    hline(s, color, x - i, y, x + i);
                }
                oj = j;
            }
            ix = ix + iy / rx;
            iy = iy - ix / rx;
        } while (i > h);
    } else {
        ix = 0;
        iy = ry * 64;
        do {
            h = (ix + 32) >> 6;
            i = (iy + 32) >> 6;
            j = (h * rx) / ry;
            k = (i * rx) / ry;
            if ((oi != i) && (oh != i)) {
                if (i) {
                    hline(s, color, x - j, y + i, x + j);
                    hline(s, color, x - j, y - i, x + j);
                } else {
                    hline(s, color, x - j, y, x + j);
                }
                oi = i;
            }
            if ((oh != h) && (oi != h) && (i != h)) {
                if (h) {
                    hline(s, color, x - k, y + h, x + k);
                    hline(s, color, x - k, y - h, x + k);
                } else {
                    hline(s, color, x - k, y, x + k);
                }
                oh = h;
            }
            ix = ix + iy / ry;
            iy = iy - ix / ry;
        } while (i > h);
    }
}

/* CPython Random.choice(seq) with len(seq) == n: seq[_randbelow(n)] */
static int pr_choice(pyrand *r, int n) {
    int k = 0;
    while ((1 << k) <= n) ++k; /* n.bit_length() */
    int v = (int)(pr_u32(r) >> (32 - k));
    while (v >= n) v = (int)(pr_u32(r) >> (32 - k));
    return v;
}

void tgo_choice_seq(uint64_t seed, int n, int count, int32_t *out) {
    pyrand r;
    pr_seed(&r, seed);
    for (int i = 0; i < count; ++i) out[i] = pr_choice(&r, n);
}

/* the handle drawing of draw_object (DR/:257-266): returns -1 if the shaft leaves the
 * surface (not supported), sets *nearint if an end point lands within 1e-9 of an integer */
static int draw_handle(surf *s, const gobj *o, const surf *base, int *nearint) {
    const double pi = 3.141592653589793; /* math.pi */
    const double angle = ((pi / 2.0) * o->angle) + pi / 4.0;
    const double r = YSCALE * 0.75;
    const double sx = o->x + XSCALE / 2.0, sy = (double)(o->y + YSCALE);
    const double ex = sx + (r * cos(angle)), ey = sy - (r * sin(angle));
    if (fabs(ex - rint(ex)) < 1e-9 || fabs(ey - rint(ey)) < 1e-9) *nearint = 1;
    int pts[4] = {(int)sx, (int)sy, (int)ex, (int)ey}; /* pg_IntFromObj truncates floats */
    if (clip_and_draw_line_width(s, 0x2F4F4Fu /* (47, 79, 79) */, 5, pts)) return -1;
    fillellipse(s, pts[2], pts[3], XSCALE / 10, XSCALE / 10, 0xFF0000u); /* int(xscale / 10) */
    blit(s, base, o->x, o->y, 0);
    return 0;
}

/* Render env e's current state: rgb [H*48][W*48][3].  Returns 0, -1 (unsupported geometry),
 * or 1 (an end point near an integer: libm watch). */
int tgo_render(const tgo_env *e, const uint8_t *sprites_rgba, int sw, int sh, uint8_t *rgb) {
    const int W = e->W * XSCALE, H = e->H * YSCALE;
    surf spr[TGO_SPR_COUNT], src;
    uint32_t *mem = (uint32_t *)malloc(sizeof(uint32_t) *
                                       ((size_t)TGO_SPR_COUNT * XSCALE * YSCALE + (size_t)W * H + (size_t)sw * sh));
    if (!mem) return -1;
    surf screen = {W, H, mem};
    src.w = sw, src.h = sh, src.px = mem + (size_t)W * H;
    for (int k = 0; k < TGO_SPR_COUNT; ++k) { /* image.load().convert_alpha(); transform.scale */
        const uint8_t *p = sprites_rgba + (size_t)k * sw * sh * 4;
        for (int i = 0; i < sw * sh; ++i)
            src.px[i] = ((uint32_t)p[4 * i + 3] << 24) | ((uint32_t)p[4 * i] << 16) |
                        ((uint32_t)p[4 * i + 1] << 8) | p[4 * i + 2];
        spr[k].w = XSCALE, spr[k].h = YSCALE;
        spr[k].px = mem + (size_t)W * H + (size_t)sw * sh + (size_t)k * XSCALE * YSCALE;
        stretch(&src, &spr[k]);
    }
    /* draw_domain (DR/:136-163) */
    pyrand rg;
    pr_seed(&rg, 12); /* self.random_generator.seed(self.seed) */
    memset(screen.px, 0, sizeof(uint32_t) * (size_t)W * H); /* fill((0, 0, 0)) */
    const tgo_level *lv = e->lv;
    for (int i = 0; i < lv->H; ++i)
        for (int j = 0; j < lv->W; ++j) {
            const char c = lv->desc[i][j];
            if (c == C_WALL) {
                int key = TGO_SPR_WALL;
                if (i > 0 && lv->desc[i - 1][j] != C_WALL) key = TGO_SPR_FLOOR;
                blit(&screen, &spr[key + pr_choice(&rg, 5)], j * XSCALE, i * YSCALE, 0);
            } else if (c == C_LADDER) {
                blit(&screen, &spr[TGO_SPR_LADDER], j * XSCALE, i * YSCALE, 0);
            } else if (c == C_OPEN) {
                blit(&screen, &spr[TGO_SPR_BACKGROUND + pr_choice(&rg, 5)], j * XSCALE, i * YSCALE, 0);
            }
        }
    int rc = 0, nearint = 0;
    for (int i = 0; i < e->nobj && !rc; ++i) { /* draw_object (DR/:238-269) */
        const gobj *o = &e->obj[i];
        if (o->x < 0) continue;
        switch (o->type) {
        case O_DOOR:
            blit(&screen, &spr[o->closed ? TGO_SPR_DOOR_CLOSED : TGO_SPR_DOOR_OPEN], o->x, o->y, 0);
            break;
        case O_KEY: blit(&screen, &spr[TGO_SPR_KEY], o->x, o->y, 0); break;
        case O_GOLD: blit(&screen, &spr[TGO_SPR_GOLD], o->x, o->y, 0); break;
        case O_BOLT:
            blit(&screen, &spr[o->locked ? TGO_SPR_BOLT_LOCKED : TGO_SPR_BOLT_OPEN], o->x, o->y, 0);
            break;
        case O_HANDLE: rc = draw_handle(&screen, o, &spr[TGO_SPR_HANDLE_BASE], &nearint); break;
        }
    }
    /* the hero at (playerx - xscale / 2, playery), flipped when facing left (DR/:157-161) */
    blit(&screen, &spr[TGO_SPR_HERO], (int)(e->playerx - XSCALE / 2.0), e->playery, !e->facing_right);
    for (size_t p = 0; p < (size_t)W * H; ++p) {
        rgb[3 * p] = (uint8_t)(screen.px[p] >> 16);
        rgb[3 * p + 1] = (uint8_t)(screen.px[p] >> 8);
        rgb[3 * p + 2] = (uint8_t)screen.px[p];
    }
    free(mem);
    return rc ? -1 : nearint;
}

/* Frames of listed envs after `steps` env-steps of the tgo_run action stream (same seeding,
 * policy and auto-reset): frames [n][H*48][W*48][3].  Returns the OR of tgo_render codes
 * (-1 on any failure). */
int tgo_run_render(const tgo_level *lv, uint64_t seed_base, const int64_t *envs, int64_t n,
                   int steps, uint64_t action_seed, int policy, int autoreset,
                   const uint8_t *sprites_rgba, int sw, int sh, uint8_t *frames, int nthreads) {
    int err = 0, warn = 0;
    const size_t fb = (size_t)lv->W * XSCALE * lv->H * YSCALE * 3;
#ifdef _OPENMP
    if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads) reduction(| : err, warn)
#endif
    for (int64_t i = 0; i < n; i++) {
        const uint64_t g = (uint64_t)envs[i];
        tgo_env *e = (tgo_env *)malloc(sizeof(tgo_env));
        if (!e) {
            err |= 1;
            continue;
        }
        env_init(e, lv, seed_base + g, NULL);
        for (int t = 0; t < steps; t++) {
            unsigned m = policy ? tgo_mask(e) : 0;
            int a = tgo_pick_action(action_seed, g, (uint64_t)t, policy, m);
            uint8_t d;
            if (tgo_step(e, a, NULL, NULL, NULL, &d)) err |= 1;
            if (autoreset && d) tgo_reset(e, NULL);
        }
        const int rc = tgo_render(e, sprites_rgba, sw, sh, frames + (size_t)i * fb);
        if (rc < 0) err |= 1;
        if (rc > 0) warn |= 1;
        free(e);
    }
    return err ? -1 : warn;
}
