// qps_native.cpp -- aggregate queries/s of concurrent callers on one table through the C ABI alone (no Python, no
// GIL): what a JNI caller, one Pinot query worker thread per query (BaseCombineOperator.java:85-115), sees.
//
//   tools/qps_native [--segments S] [--docs N] [--seconds T] [--threads 1,2,4,8] [--no-cache]
//
// The C1 table (dim U[0,16), filt U[0,1000), metric U[0,10000)) is generated on the device; every
// thread runs "SELECT SUM(metric) FROM t WHERE filt BETWEEN 250 AND 749 GROUP BY dim" on its own HIP stream
// (pgpu_execute_groupby: plan + execute + finalize) and checks each result against the first one.  One JSON line.
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../include/pinotgpu.h"

static void check(int rc, const char* what) {
  if (rc == 0) return;
  char buf[512];
  pgpu_last_error(buf, sizeof buf);
  fprintf(stderr, "%s failed (%d): %s\n", what, rc, buf);
  exit(1);
}

int main(int argc, char** argv) {
  int segments = 1, docs = 1000000;
  double seconds = 3.0;
  bool no_cache = false;
  std::vector<int> thread_counts = {1, 2, 4, 8};
  for (int i = 1; i < argc; ++i) {
    const std::string a = argv[i];
    if (a == "--segments" && i + 1 < argc) segments = atoi(argv[++i]);
    else if (a == "--docs" && i + 1 < argc) docs = atoi(argv[++i]);
    else if (a == "--seconds" && i + 1 < argc) seconds = atof(argv[++i]);
    else if (a == "--no-cache") no_cache = true;
    else if (a == "--threads" && i + 1 < argc) {
      thread_counts.clear();
      for (char* s = strtok(argv[++i], ","); s; s = strtok(nullptr, ",")) thread_counts.push_back(atoi(s));
    }
  }
  const char* names[3] = {"dim", "filt", "metric"};
  const int32_t types[3] = {PGPU_INT, PGPU_INT, PGPU_INT};
  pgpu_table t = nullptr;
  check(pgpu_table_create(0, 3, names, types, &t), "pgpu_table_create");
  pgpu_gen_column gen[3];
  memset(gen, 0, sizeof gen);
  const int64_t hi[3] = {16, 1000, 10000};
  for (int c = 0; c < 3; ++c) {
    gen[c].kind = PGPU_GEN_UNIFORM;
    gen[c].column_index = c;
    gen[c].lo = 0;
    gen[c].hi = hi[c];
  }
  std::vector<int64_t> handles(segments);
  for (int s = 0; s < segments; ++s)
    check(pgpu_generate_segment(t, gen, 3, (int64_t)s * docs, docs, &handles[s]), "pgpu_generate_segment");

  const char* range[2] = {"250", "749"};
  pgpu_predicate pred;
  memset(&pred, 0, sizeof pred);
  pred.type = PGPU_PRED_RANGE;
  pred.column = 1;
  pred.num_values = 2;
  pred.lower_inclusive = 1;
  pred.upper_inclusive = 1;
  pred.values = range;
  const pgpu_filter_op filter[1] = {{PGPU_OP_PRED, 0}};
  const int32_t group_by[1] = {0};
  const pgpu_agg aggs[1] = {{PGPU_AGG_SUM, 2}};
  pgpu_query q;
  memset(&q, 0, sizeof q);
  q.num_predicates = 1;
  q.predicates = &pred;
  q.num_filter_ops = 1;
  q.filter = filter;
  q.num_group_by = 1;
  q.group_by = group_by;
  q.num_aggs = 1;
  q.aggs = aggs;
  q.num_groups_limit = 100000;
  q.options = no_cache ? PGPU_OPT_NO_PLAN_CACHE : 0;

  // the reference answer
  pgpu_result r0 = nullptr;
  check(pgpu_execute_groupby(t, handles.data(), segments, &q, nullptr, &r0), "pgpu_execute_groupby");
  int64_t n0 = 0;
  check(pgpu_result_num_groups(r0, &n0), "pgpu_result_num_groups");
  std::vector<int64_t> ref(n0 > 0 ? n0 : 1);
  check(pgpu_result_values_i64(r0, 0, ref.data()), "pgpu_result_values_i64");
  pgpu_result_destroy(r0);

  printf("{\"workload\": \"c1\", \"segments\": %d, \"docs_per_segment\": %d, \"plan_cache\": %s, \"groups\": %lld, "
         "\"runs\": [", segments, docs, no_cache ? "false" : "true", (long long)n0);
  for (size_t k = 0; k < thread_counts.size(); ++k) {
    const int T = thread_counts[k];
    std::atomic<bool> stop{false};
    std::atomic<int64_t> bad{0};
    std::vector<int64_t> done(T, 0);
    std::vector<std::thread> th;
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < T; ++i)
      th.emplace_back([&, i] {
        hipStream_t s;
        if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) { bad++; return; }
        std::vector<int64_t> v(ref.size());
        while (!stop.load(std::memory_order_relaxed)) {
          pgpu_result r = nullptr;
          if (pgpu_execute_groupby(t, handles.data(), segments, &q, s, &r)) { bad++; break; }
          int64_t n = 0;
          pgpu_result_num_groups(r, &n);
          if (n != n0 || pgpu_result_values_i64(r, 0, v.data()) || memcmp(v.data(), ref.data(), n * 8)) bad++;
          pgpu_result_destroy(r);
          ++done[i];
        }
        (void)hipStreamDestroy(s);
      });
    std::this_thread::sleep_for(std::chrono::duration<double>(seconds));
    stop = true;
    for (auto& x : th) x.join();
    const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    int64_t total = 0;
    for (int64_t d : done) total += d;
    printf("%s{\"threads\": %d, \"queries\": %lld, \"seconds\": %.3f, \"qps\": %.1f, \"rows_per_s\": %.4g, "
           "\"results_match\": %s}", k ? ", " : "", T, (long long)total, el, total / el,
           total / el * segments * (double)docs, bad.load() ? "false" : "true");
    fflush(stdout);
  }
  printf("]}\n");
  pgpu_table_destroy(t);
  return 0;
}
