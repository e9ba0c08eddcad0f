// madnn host runtime (C++17, no GPU code): the planner's hot combinatorics and
// the pipeline scheduler, exposed through a C ABI for ctypes.
//
//  * madnn_partition      — contiguous layer->stage partition minimising the
//                            bottleneck stage cost under a per-stage memory cap
//                            (the auto-partitioner's core).  The
//                            reference has no partitioner: its only planning is
//                            the sync-period heuristic (datamodule.lua:68-78).
//  * madnn_plan_buckets   — gradient bucket assignment in backward-ready order
//                            with 16-element alignment so every tensor of a
//                            bucket starts on a 16-byte boundary for the K4
//                            vector path (replaces datamodule.lua:211-224's
//                            one-collective-per-tensor loop).
//  * madnn_pipeline_order — per-rank compute order of GPipe / 1F1B / interleaved
//                            1F1B pipelines; the engine derives all
//                            communication from it.
//  * madnn_hash_*         — collective-order fingerprint used by the debug
//                            checker to catch rank divergence.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <limits>
#include <vector>

extern "C" {

// costs[L], mems[L]: per-layer time and bytes.  Writes bounds[S+1] with
// bounds[0] = 0, bounds[S] = L.  Returns the bottleneck cost, or -1 if no
// partition satisfies mem_cap (mem_cap <= 0 disables the cap).
double madnn_partition(const double* costs, const double* mems, int L, int S, double mem_cap, int* bounds) {
  if (L <= 0 || S <= 0 || S > L) return -1.0;
  std::vector<double> pc(L + 1, 0.0), pm(L + 1, 0.0);
  for (int i = 0; i < L; ++i) {
    pc[i + 1] = pc[i] + costs[i];
    pm[i + 1] = pm[i] + (mems ? mems[i] : 0.0);
  }
  const double INF = std::numeric_limits<double>::infinity();
  // dp[s][j]: best bottleneck for the first j layers in s stages.
  std::vector<std::vector<double>> dp(S + 1, std::vector<double>(L + 1, INF));
  std::vector<std::vector<int>> arg(S + 1, std::vector<int>(L + 1, -1));
  dp[0][0] = 0.0;
  for (int s = 1; s <= S; ++s) {
    for (int j = s; j <= L - (S - s); ++j) {
      for (int i = s - 1; i < j; ++i) {
        if (dp[s - 1][i] == INF) continue;
        const double mem = pm[j] - pm[i];
        if (mem_cap > 0 && mem > mem_cap) continue;
        const double c = std::max(dp[s - 1][i], pc[j] - pc[i]);
        // tie-break toward balanced prefix (smaller last stage first)
        if (c < dp[s][j] - 1e-12) {
          dp[s][j] = c;
          arg[s][j] = i;
        }
      }
    }
  }
  if (dp[S][L] == INF) return -1.0;
  int j = L;
  bounds[S] = L;
  for (int s = S; s >= 1; --s) {
    int i = arg[s][j];
    bounds[s - 1] = i;
    j = i;
  }
  return dp[S][L];
}

// numels[n] in backward-ready order; cap_elems per bucket (>= 1).  Writes
// bucket_of[n], offset_of[n] (element offset in its bucket, 16-aligned) and
// bucket_size[n] (padded element count per bucket, only the first nb used).
// Returns the number of buckets.
int madnn_plan_buckets(const int64_t* numels, int n, int64_t cap_elems, int align, int* bucket_of,
                       int64_t* offset_of, int64_t* bucket_size) {
  if (align < 1) align = 1;
  int b = 0;
  int64_t cur = 0;
  bool empty = true;
  for (int i = 0; i < n; ++i) {
    const int64_t ne = numels[i];
    const int64_t padded = (ne + align - 1) / align * align;
    if (!empty && cur + padded > cap_elems) {
      bucket_size[b] = cur;
      ++b;
      cur = 0;
      empty = true;
    }
    bucket_of[i] = b;
    offset_of[i] = cur;
    cur += padded;
    empty = false;
  }
  if (!empty) {
    bucket_size[b] = cur;
    ++b;
  }
  return b;
}

// Per-rank COMPUTE order of a (possibly interleaved) pipeline as (op, chunk, microbatch)
// triples, op 0 = forward, 1 = backward.  Communication is not part of the order: every
// message travels on a one-directional FIFO channel (activations r -> r+1, gradients
// r+1 -> r, plus the two ring edges S-1 -> 0 / 0 -> S-1 of the interleaved layout), and
// the orders below make every channel's send order equal its receive order, so the engine
// can post receives ahead of time and never wait on a send.
//   kind 0 GPipe: all forwards, then all backwards (V = 1).
//   kind 1 1F1B (PipeDream-flush, V = 1): S-s-1 warm-up forwards, then F/B pairs.
//   kind 2 interleaved 1F1B with V model chunks per rank; chunk c of rank s is virtual
//          stage c*S + s.  Forward step k runs chunk (k mod SV) / S on microbatch
//          (k / SV) * S + k mod S; backward step k runs chunk V-1-(k mod SV)/S on the same
//          microbatch formula; warm-up = 2(S-s-1) + (V-1)S forwards.  Needs M % S == 0.
// Returns the number of triples (2*M*V), or -1 on invalid arguments.
int madnn_pipeline_order(int kind, int stage, int nstages, int nmicro, int nchunks, int* out) {
  if (nstages <= 0 || stage < 0 || stage >= nstages || nmicro <= 0 || nchunks <= 0) return -1;
  int k = 0;
  auto emit = [&](int op, int c, int m) {
    out[3 * k] = op;
    out[3 * k + 1] = c;
    out[3 * k + 2] = m;
    ++k;
  };
  if (kind == 0 || kind == 1) {
    if (nchunks != 1) return -1;
    if (kind == 0) {
      for (int m = 0; m < nmicro; ++m) emit(0, 0, m);
      for (int m = 0; m < nmicro; ++m) emit(1, 0, m);
      return k;
    }
    const int warm = std::min(nstages - stage - 1, nmicro);
    int f = 0, b = 0;
    for (int i = 0; i < warm; ++i) emit(0, 0, f++);
    while (f < nmicro) {
      emit(0, 0, f++);
      emit(1, 0, b++);
    }
    while (b < nmicro) emit(1, 0, b++);
    return k;
  }
  if (kind != 2 || nmicro % nstages != 0) return -1;
  const int S = nstages, V = nchunks, SV = S * V, total = nmicro * V;
  auto mb = [&](int step) { return (step / SV) * S + step % S; };
  auto fchunk = [&](int step) { return (step % SV) / S; };
  const int warm = std::min(2 * (S - stage - 1) + (V - 1) * S, total);
  int f = 0, b = 0;
  for (; f < warm; ++f) emit(0, fchunk(f), mb(f));
  while (f < total) {
    emit(0, fchunk(f), mb(f));
    ++f;
    emit(1, V - 1 - fchunk(b), mb(b));
    ++b;
  }
  for (; b < total; ++b) emit(1, V - 1 - fchunk(b), mb(b));
  return k;
}

// 64-bit FNV-1a over (op, group, numel, dtype) events.
uint64_t madnn_hash_init() { return 1469598103934665603ULL; }

uint64_t madnn_hash_event(uint64_t h, int op, int group, int64_t numel, int dtype) {
  const int64_t words[4] = {op, group, numel, dtype};
  const unsigned char* p = reinterpret_cast<const unsigned char*>(words);
  for (size_t i = 0; i < sizeof(words); ++i) {
    h ^= p[i];
    h *= 1099511628211ULL;
  }
  return h;
}

}  // extern "C"
