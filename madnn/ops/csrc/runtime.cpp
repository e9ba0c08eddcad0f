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
//  * madnn_pipeline_schedule — GPipe / 1F1B action lists per stage.
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

// Action encoding: op * 1'000'000 + microbatch, op 0 = forward, 1 = backward.
// kind 0 = GPipe (all F then all B), kind 1 = 1F1B (PipeDream-flush).
// Writes 2*M actions into out; returns the count.
int madnn_pipeline_schedule(int kind, int stage, int nstages, int nmicro, int* out) {
  int k = 0;
  if (kind == 0) {
    for (int m = 0; m < nmicro; ++m) out[k++] = m;
    for (int m = 0; m < nmicro; ++m) out[k++] = 1000000 + m;
    return k;
  }
  const int warm = std::min(nstages - stage - 1, nmicro);
  int f = 0, b = 0;
  for (int i = 0; i < warm; ++i) out[k++] = f++;
  while (f < nmicro) {
    out[k++] = f++;
    out[k++] = 1000000 + b++;
  }
  while (b < nmicro) out[k++] = 1000000 + b++;
  return k;
}

// Full per-stage pipeline PROGRAM, communication included, as (op, a, b)
// triples.  Ops: 0 RECV_FWD m | 1 FWD m | 2 SEND_FWD m | 3 RECV_BWD m | 4 BWD m |
// 5 SEND_BWD m | 6 SEND_FWD_RECV_BWD (send m=a, recv m=b) |
// 7 SEND_BWD_RECV_FWD (send m=a, recv m=b).
// 1F1B follows the non-interleaved PipeDream-flush order with the steady-state
// send/recv pairs batched into one group, which is what keeps two adjacent
// stages from both blocking in a send on a shared point-to-point channel.
// Returns the number of triples written (<= 6*M: GPipe; 1F1B <= 4*M + 1).
int madnn_pipeline_program(int kind, int stage, int nstages, int nmicro, int* out) {
  int k = 0;
  auto emit = [&](int op, int a, int b) {
    out[3 * k] = op;
    out[3 * k + 1] = a;
    out[3 * k + 2] = b;
    ++k;
  };
  if (kind == 0) {  // GPipe
    for (int m = 0; m < nmicro; ++m) { emit(0, m, -1); emit(1, m, -1); emit(2, m, -1); }
    for (int m = 0; m < nmicro; ++m) { emit(3, m, -1); emit(4, m, -1); emit(5, m, -1); }
    return k;
  }
  const int warm = std::min(nstages - stage - 1, nmicro);
  const int steady = nmicro - warm;
  for (int i = 0; i < warm; ++i) { emit(0, i, -1); emit(1, i, -1); emit(2, i, -1); }
  if (steady > 0) emit(0, warm, -1);
  for (int i = 0; i < steady; ++i) {
    const int f = warm + i;
    emit(1, f, -1);
    emit(6, f, i);
    emit(4, i, -1);
    if (i == steady - 1) emit(5, i, -1);
    else emit(7, i, f + 1);
  }
  for (int i = steady; i < nmicro; ++i) { emit(3, i, -1); emit(4, i, -1); emit(5, i, -1); }
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
