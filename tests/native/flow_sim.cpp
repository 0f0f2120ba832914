// CPU model of k_flow's work protocol (gym-treasure-game_amd/csrc/tg_flow.h), threads for waves
// and seq_cst atomics for the device's: the step-0 deal, (step, option) lists filled per 64-entry
// chunk and pushed by the writer that completes one, the partial chunks flushed by the last
// classification of a step, run items by ticket, per-chunk outstanding counts, and the chunks a
// run item completes (the first classified by its wave, the rest pushed as classify items).
// Checks: every chunk classified exactly once per step, every env run exactly once per step it
// runs in, termination.  Test infrastructure (tests/test_flow_protocol.py), not the product.
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <thread>
#include <vector>

constexpr int NLIST = 10, KMAX = 16, QCLS = 15;
constexpr unsigned EMPTY = 0xFFFFFFFFu;
struct Sub {
  std::atomic<int> init{0}, qhead{0}, qtail{0}, fin{0}, done{0};
  std::atomic<int> cls[KMAX];
  std::atomic<int> ltail[KMAX * NLIST];
  std::vector<std::atomic<int>> fill, list;
  std::vector<std::atomic<unsigned>> q;
};
int N, C, P, K, jcap, lcap, qcap;
std::vector<std::atomic<int>> outst, ccount, rcount;
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

void wave(int x, int seed, int runpct) {
  Sub* S = subs[x];
  std::mt19937 rng(seed);
  const int Cx = (C - x + P - 1) / P;
  if (Cx <= 0) return;  // a batch of fewer chunks than sub-problems (as k_flow)
  auto push = [&](unsigned item) {
    const int at = S->qtail.fetch_add(1);
    if (at >= qcap) { errors++; fprintf(stderr, "queue overflow\n"); return; }
    S->q[at].store(item);
  };
  auto classify = [&](int c, int t) -> int {
    if (ccount[(size_t)c * K + t].fetch_add(1) != 0) { errors++; fprintf(stderr, "dup classify c %d t %d\n", c, t); }
    int bk[64], cnt = 0;
    for (int l = 0; l < 64; ++l) {
      const int i = c * 64 + l;
      bk[l] = i < N ? opt_of(i, t, runpct) : -1;
      cnt += bk[l] >= 0;
    }
    if (cnt) outst[c].store(cnt);
    for (int k = 0; k < NLIST && cnt; ++k) {
      int nb = 0;
      for (int l = 0; l < 64; ++l) nb += bk[l] == k;
      if (!nb) continue;
      const int lidx = t * NLIST + k;
      const int base = S->ltail[lidx].fetch_add(nb);
      int r = 0;
      for (int l = 0; l < 64; ++l)
        if (bk[l] == k) S->list[(size_t)lidx * lcap + base + r++].store(c * 64 + l);
      const int j0 = base >> 6, in0 = std::min(nb, 64 - (base & 63));
      if (S->fill[(size_t)lidx * jcap + j0].fetch_add(in0) + in0 == 64) push((unsigned)(t << 28 | k << 24 | j0));
      if (nb > in0 && S->fill[(size_t)lidx * jcap + j0 + 1].fetch_add(nb - in0) + (nb - in0) == 64)
        push((unsigned)(t << 28 | k << 24 | (j0 + 1)));
    }
    if (S->cls[t].fetch_add(1) + 1 == Cx)  // the step's last classification: partial chunks
      for (int k = 0; k < NLIST; ++k) {
        const int tail = S->ltail[t * NLIST + k].load();
        if (tail & 63) push((unsigned)(t << 28 | k << 24 | (tail >> 6)));
      }
    return cnt;
  };
  bool phase0 = true;
  int cc = -1, ct = 0;
  const auto t_start = std::chrono::steady_clock::now();
  while (true) {
    int c, t;
    if (cc >= 0) {
      c = cc; t = ct; cc = -1;
    } else if (phase0) {
      const int j = S->init.fetch_add(1);
      if (j >= Cx) { phase0 = false; continue; }
      c = x + P * j; t = 0;
    } else {
      const int h = S->qhead.fetch_add(1);
      unsigned item = EMPTY;
      while (true) {
        if (h < qcap) item = S->q[h].load();
        if (item != EMPTY || S->done.load()) break;
        if (std::chrono::steady_clock::now() - t_start > std::chrono::seconds(20)) {
          errors++; fprintf(stderr, "wait bound\n"); S->done.store(1); break;
        }
        std::this_thread::yield();
      }
      if (item == EMPTY) break;
      t = (int)(item >> 28);
      const int k = (int)((item >> 24) & 15u);
      if (k == QCLS) {
        c = (int)(item & 0xFFFFFFu);
      } else {  // a run item
        const int j = (int)(item & 0xFFFFFFu), lidx = t * NLIST + k;
        const int m = std::min(64, S->ltail[lidx].load() - 64 * j);
        if (S->fill[(size_t)lidx * jcap + j].load() != m) { errors++; fprintf(stderr, "fill mismatch\n"); }
        std::vector<int> envs;
        for (int l = 0; l < m; ++l) envs.push_back(S->list[(size_t)lidx * lcap + 64 * j + l].load());
        if (rng() % 4 == 0) std::this_thread::sleep_for(std::chrono::microseconds(rng() % 200));
        std::vector<int> ready;
        for (int i : envs) {
          if (rcount[(size_t)i * K + t].fetch_add(1) != 0) { errors++; fprintf(stderr, "dup run\n"); }
          if (opt_of(i, t, runpct) != k) { errors++; fprintf(stderr, "wrong list\n"); }
          if (outst[i >> 6].fetch_sub(1) == 1) ready.push_back(i >> 6);
        }
        if (ready.empty()) continue;
        ++t;
        if (t >= K) {
          const int nr = (int)ready.size();
          if (S->fin.fetch_add(nr) + nr == Cx) S->done.store(1);
          continue;
        }
        c = ready[0];
        for (size_t r = 1; r < ready.size(); ++r) push((unsigned)(t << 28 | QCLS << 24 | ready[r]));
      }
    }
    if (t >= K) {
      if (S->fin.fetch_add(1) + 1 == Cx) S->done.store(1);
      continue;
    }
    if (classify(c, t) == 0) { cc = c; ct = t + 1; }
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
  lcap = cxm * 64; jcap = cxm + 1; qcap = KMAX * (2 * cxm + NLIST);  // as tg_amd.hip flow_init
  outst = std::vector<std::atomic<int>>(C);
  ccount = std::vector<std::atomic<int>>((size_t)C * K);
  rcount = std::vector<std::atomic<int>>((size_t)N * K);
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
  for (int c = 0; c < C; ++c)
    for (int t = 0; t < K; ++t) miss += ccount[(size_t)c * K + t].load() != 1;
  for (int i = 0; i < N; ++i)
    for (int t = 0; t < K; ++t) {
      want += opt_of(i, t, runpct) >= 0;
      runs += rcount[(size_t)i * K + t].load();
    }
  printf("N %d K %d P %d W %d run %d%%: errors %d, chunk-steps not classified once %ld, runs %ld / %ld\n",
         N, K, P, W, runpct, errors.load(), miss, runs, want);
  return errors.load() || miss || runs != want;
}
