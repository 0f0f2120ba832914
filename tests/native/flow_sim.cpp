// CPU model of k_flow's work protocol (gym-treasure-game_amd/csrc/tg_flow.h, round 6's chunk
// rounds), threads for waves and seq_cst atomics for the device's: rounds of 64-env chunks (the
// first dealt out by a counter), in which each env not yet past step K - 1 runs ahead from its
// own next step, finished in place while its option cannot run, until it is listed at (t', k);
// (step, option) lists filled per 64-entry chunk and pushed by the writer that completes one;
// per-step counts of classified envs, the wave that completes a step's count sealing its
// partial chunks; run items by ticket, each env's next step recorded and its chunk's
// outstanding count decremented, the chunks a run item readies given their next round (the
// first by its wave, the rest pushed as classify items); a waiting wave first in line seals the
// fullest partial chunk of the lowest open steps.  Checks: every env-step classified exactly
// once, every env run exactly once per step it runs in, fill counts equal to the entries run,
// termination.  Test infrastructure (tests/test_flow_protocol.py), not the product.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <thread>
#include <vector>

constexpr int NLIST = 10, KMAX = 16;
constexpr unsigned EMPTY = 0xFFFFFFFFu;
struct Sub {
  std::atomic<int> init{0}, qhead{0}, qtail{0}, fin{0}, done{0};
  std::atomic<int> cls[KMAX];
  std::atomic<int> ltail[KMAX * NLIST];
  std::vector<std::atomic<int>> fill, list;
  std::vector<std::atomic<unsigned>> q;
};
int N, C, P, K, jcap, lcap, qcap, seal_below;
constexpr int QCLS = 15;
std::vector<std::atomic<int>> ccount, rcount, outst, cstep;
std::atomic<int> errors{0};
std::vector<Sub*> subs;

int opt_of(int i, int t, int runpct) {  // -1 (no run) or the env's list at step t
  unsigned h = (unsigned)i * 2654435761u ^ (unsigned)(t + 1) * 40503u;
  h ^= h >> 13;
  h *= 0x5bd1e995u;
  h ^= h >> 15;
  if ((int)(h % 100) >= runpct) return -1;
  return (int)((h >> 8) % NLIST);
}
int envs_of(int x) {  // tg_flow.h flow_envs
  const int Cx = (C - x + P - 1) / P;
  return Cx <= 0 ? 0 : Cx * 64 - ((C - 1) % P == x ? C * 64 - N : 0);
}

void wave(int x, int seed, int runpct) {
  Sub* S = subs[x];
  std::mt19937 rng(seed);
  const int Cx = (C - x + P - 1) / P;
  if (Cx <= 0) return;  // a batch of fewer chunks than sub-problems (as k_flow)
  const int nx = envs_of(x);
  auto push = [&](int t, int k, int j, int cnt) {
    const int at = S->qtail.fetch_add(1);
    if (at >= qcap) { errors++; fprintf(stderr, "queue overflow\n"); return; }
    S->q[at].store((unsigned)(t << 28 | k << 24 | (cnt - 1) << 18 | j));
  };
  auto fill_add = [&](int t, int k, int j, int add) {  // tg_flow.h fill_add
    if (j >= jcap) { errors++; fprintf(stderr, "jcap\n"); return; }
    const int nv = S->fill[(size_t)(t * NLIST + k) * jcap + j].fetch_add(add) + add;
    if ((nv & 0xFF) == 64) push(t, k, j, (nv >> 8) ? (nv >> 8) : 64);
  };
  auto seal = [&](int t, int k, bool reserve) {  // tg_flow.h seal
    std::atomic<int>& lt = S->ltail[t * NLIST + k];
    int v = lt.load();
    if (!(v & 63) || (reserve && (v >> 6) >= seal_below)) return;
    if (!lt.compare_exchange_strong(v, (v | 63) + 1)) return;
    const int r = v & 63;
    fill_add(t, k, v >> 6, (64 - r) + (r << 8));
  };
  // a round of chunk c (k_flow round): returns the envs listed
  auto round = [&](int c, bool first) -> int {
    std::vector<int> envs, from;
    for (int l = 0; l < 64; ++l) {
      const int i = c * 64 + l;
      if (i >= N) continue;
      const int t = first ? 0 : cstep[i].load();
      if (t < K) { envs.push_back(i); from.push_back(t); }
    }
    const int m = (int)envs.size();
    std::vector<int> tl(m), kl(m, -1), pos(m);
    int cnt = 0;
    for (int l = 0; l < m; ++l) {
      int t = from[l];
      for (; t < K; ++t) {
        if (ccount[(size_t)envs[l] * K + t].fetch_add(1) != 0) {
          errors++; fprintf(stderr, "dup classify i %d t %d\n", envs[l], t);
        }
        if ((kl[l] = opt_of(envs[l], t, runpct)) >= 0) break;
      }
      tl[l] = t;
      cnt += t < K;
    }
    for (int l = 0; l < m; ++l)  // reserve, write the entry ...
      if (tl[l] < K) {
        const int lidx = tl[l] * NLIST + kl[l];
        pos[l] = S->ltail[lidx].fetch_add(1);
        if (pos[l] >= lcap) { errors++; fprintf(stderr, "lcap\n"); tl[l] = K; continue; }
        S->list[(size_t)lidx * lcap + pos[l]].store(envs[l]);
      } else {
        cstep[envs[l]].store(K);
      }
    if (cnt) outst[c].store(cnt);
    if (rng() % 8 == 0) std::this_thread::sleep_for(std::chrono::microseconds(rng() % 100));
    for (int l = 0; l < m; ++l)  // ... then the fill counts (the completing writer pushes)
      if (tl[l] < K) fill_add(tl[l], kl[l], pos[l] >> 6, 1);
    for (int sp = 0; sp < K; ++sp) {  // steps classified: from .. min(tl, K - 1)
      int cs = 0;
      for (int l = 0; l < m; ++l) cs += from[l] <= sp && sp <= std::min(tl[l], K - 1);
      if (cs && S->cls[sp].fetch_add(cs) + cs == nx)
        for (int k = 0; k < NLIST; ++k) seal(sp, k, false);  // the step's partial chunks
    }
    return cnt;
  };
  bool deal = true;
  const auto t_start = std::chrono::steady_clock::now();
  while (true) {
    int c;
    bool first = false;
    if (deal) {
      const int j = S->init.fetch_add(1);
      if (j >= Cx) { deal = false; continue; }
      c = x + P * j;
      first = true;
    } else {
      const int h = S->qhead.fetch_add(1);
      unsigned item = EMPTY;
      int polls = 0;
      while (true) {
        if (h < qcap) item = S->q[h].load();
        if (item != EMPTY || S->done.load()) break;
        if (h == S->qtail.load() && ++polls % 64 == 0) {  // first in line, idle: seal
          int best = 0, bt = -1, bk = -1;  // the lowest step's fullest partial chunk
          for (int tc = 0; tc < K && bt < 0; ++tc)
            for (int kc = 0; kc < NLIST; ++kc) {
              const int v = S->ltail[tc * NLIST + kc].load();
              if ((v & 63) > best && (v >> 6) < seal_below) { best = v & 63; bt = tc; bk = kc; }
            }
          if (bt >= 0) seal(bt, bk, true);
        }
        if (std::chrono::steady_clock::now() - t_start > std::chrono::seconds(20)) {
          errors++; fprintf(stderr, "wait bound\n"); S->done.store(1); break;
        }
        std::this_thread::yield();
      }
      if (item == EMPTY) break;
      const int t = (int)(item >> 28), k = (int)((item >> 24) & 15u), j = (int)(item & 0x3FFFFu);
      if (k == QCLS) {
        c = j;
      } else {
        const int lidx = t * NLIST + k;
        const int m = (int)((item >> 18) & 63u) + 1;
        const int fv = S->fill[(size_t)lidx * jcap + j].load();
        if ((fv & 0xFF) != 64 || ((fv >> 8) ? (fv >> 8) : 64) != m) { errors++; fprintf(stderr, "fill mismatch\n"); }
        std::vector<int> envs;
        for (int l = 0; l < m; ++l) envs.push_back(S->list[(size_t)lidx * lcap + 64 * j + l].load());
        if (rng() % 4 == 0) std::this_thread::sleep_for(std::chrono::microseconds(rng() % 200));
        std::vector<int> ready;
        for (int i : envs) {
          if (i < 0 || i >= N || (i >> 6) % P != x) { errors++; fprintf(stderr, "bad entry\n"); return; }
          if (rcount[(size_t)i * K + t].fetch_add(1) != 0) { errors++; fprintf(stderr, "dup run\n"); }
          if (opt_of(i, t, runpct) != k) { errors++; fprintf(stderr, "wrong list\n"); }
          cstep[i].store(t + 1);
          if (outst[i >> 6].fetch_sub(1) == 1) ready.push_back(i >> 6);
        }
        if (ready.empty()) continue;
        c = ready[0];
        for (size_t r = 1; r < ready.size(); ++r) push(0, QCLS, ready[r], 1);
      }
    }
    if (round(c, first) == 0 && S->fin.fetch_add(1) + 1 == Cx) S->done.store(1);
  }
}

int main(int argc, char** argv) {
  N = argc > 1 ? atoi(argv[1]) : 70001;
  K = argc > 2 ? atoi(argv[2]) : 16;
  P = argc > 3 ? atoi(argv[3]) : 2;
  const int W = argc > 4 ? atoi(argv[4]) : 16;       // waves per sub-problem
  const int runpct = argc > 5 ? atoi(argv[5]) : 21;  // env-steps that run an option (%)
  C = (N + 63) / 64;
  const int cxm = (C + P - 1) / P;
  seal_below = 3 * cxm; lcap = 4 * cxm * 64; jcap = 4 * cxm + 1; qcap = KMAX * (NLIST * jcap + cxm);  // flow_init
  ccount = std::vector<std::atomic<int>>((size_t)N * K);
  rcount = std::vector<std::atomic<int>>((size_t)N * K);
  outst = std::vector<std::atomic<int>>(C);
  cstep = std::vector<std::atomic<int>>(N);
  for (int x = 0; x < P; ++x) {
    Sub* s = new Sub();
    for (auto& a : s->cls) a = 0;
    for (auto& a : s->ltail) a = 0;
    s->fill = std::vector<std::atomic<int>>((size_t)KMAX * NLIST * jcap);
    s->list = std::vector<std::atomic<int>>((size_t)KMAX * NLIST * lcap);
    s->q = std::vector<std::atomic<unsigned>>(qcap);
    for (auto& a : s->q) a = EMPTY;
    subs.push_back(s);
  }
  std::vector<std::thread> th;
  for (int x = 0; x < P; ++x)
    for (int w = 0; w < W; ++w) th.emplace_back(wave, x, x * 1000 + w, runpct);
  for (auto& t : th) t.join();
  long miss = 0, runs = 0, want = 0;
  for (int i = 0; i < N; ++i)
    for (int t = 0; t < K; ++t) {
      miss += ccount[(size_t)i * K + t].load() != 1;
      want += opt_of(i, t, runpct) >= 0;
      runs += rcount[(size_t)i * K + t].load();
    }
  printf("N %d K %d P %d W %d run %d%%: errors %d, env-steps not classified once %ld, runs %ld / %ld\n",
         N, K, P, W, runpct, errors.load(), miss, runs, want);
  return errors.load() || miss || runs != want;
}
