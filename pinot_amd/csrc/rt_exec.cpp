// rt_exec.cpp -- query execution (launches) and finalize (rt.h).
#include "rt_decls.h"

namespace pgpu {
// ---- query deadlines (BaseCombineOperator.java:79-132: the combine waits until QueryContext.getEndTimeMs and then
// returns a timeout block; GroupByCombineOperator.java:193-203 for group-by).  The persistent scans compare the
// device wall clock against the deadline converted to clock ticks and stop taking tiles past it.
double epoch_us() {
  return (double)std::chrono::duration_cast<std::chrono::microseconds>(
             std::chrono::system_clock::now().time_since_epoch()).count();
}

// Device clock ticks at host epoch time end_ms, never earlier than the true reading (the calibration pairs a clock
// value with a host time taken before the kernel that read it, so queueing delay only makes deadlines later).
int deadline_ticks(pgpu_table_s* t, int64_t end_ms, uint64_t* out) {
  std::lock_guard<std::mutex> g(t->clock_mu);
  if (!t->clock_stream) {
    int khz = 0;
    HIP_TRY(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, t->device));
    if (khz <= 0) return fail(PGPU_ERR_DEVICE, "device wall clock rate unavailable");
    t->clock_rate_khz = khz;
    HIP_TRY(hipStreamCreateWithFlags(&t->clock_stream, hipStreamNonBlocking));
    HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&t->clock_pinned), 64, hipHostMallocDefault));
  }
  const double steady = now_us();
  if (t->clock_steady_us < 0 || steady - t->clock_steady_us > 10e6) {
    double best = 1e300;
    for (int i = 0; i < 3 && best > 200.0; ++i) {  // the tightest of up to 3 readings
      const double h0 = epoch_us();
      if (launch_read_clock(t->clock_pinned, t->clock_stream))
        return fail(PGPU_ERR_DEVICE, "clock read launch failed: %s", hipGetErrorString(hipGetLastError()));
      HIP_TRY(hipStreamSynchronize(t->clock_stream));
      const double h1 = epoch_us();
      if (h1 - h0 < best) {
        best = h1 - h0;
        t->clock_host_us = h0;
        t->clock_ticks = *reinterpret_cast<volatile uint64_t*>(t->clock_pinned);
      }
    }
    t->clock_steady_us = steady;
  }
  const double dt_us = (double)end_ms * 1000.0 - t->clock_host_us;
  *out = t->clock_ticks + (dt_us > 0 ? (uint64_t)(dt_us * t->clock_rate_khz / 1000.0) : 0);
  if (*out == 0) *out = 1;
  return 0;
}

// The combine's timeout: aggregation-only plans report BaseCombineOperator's EXECUTION_TIMEOUT_ERROR (250),
// group-by plans GroupByCombineOperator's QUERY_EXECUTION_ERROR (200) wrapping a TimeoutException.
int timeout_fail(const pgpu_plan_s* P) {
  if (P->key_cols.empty())
    return fail(PGPU_ERR_TIMEOUT, "QueryException 250 (EXECUTION_TIMEOUT_ERROR): Timed out while polling results block");
  return fail(PGPU_ERR_TIMEOUT, "QueryException 200 (QUERY_EXECUTION_ERROR): Timed out while combining group-by results "
              "after %lldms", (long long)(P->end_time_ms - P->exec_start_ms));
}

// Leaves the plan's scratch to the device work still queued on `stream` (see Scratch::busy).
int abandon_scratch(Scratch* sc, hipStream_t stream) {
  if (!sc) return 0;
  if (!sc->busy) HIP_TRY(hipEventCreateWithFlags(&sc->busy, hipEventDisableTiming));
  HIP_TRY(hipEventRecord(sc->busy, stream));
  sc->abandoned = true;
  return 0;
}

// Waits for the plan's work on `stream`.  With an end time the wait gives up at it, as the combine's
// _blockingQueue.poll(endTimeMs - now) / _operatorLatch.await(timeoutMs) do (BaseCombineOperator.java:193-203,
// GroupByCombineOperator.java:193-203): the query returns PGPU_ERR_TIMEOUT at its deadline and the device work
// left running keeps its scratch out of the pool until it completes.
int cancel_fail() {
  return fail(PGPU_ERR_CANCELLED, "QueryException 503 (QUERY_CANCELLATION_ERROR): Query was cancelled");
}

bool cancelled(const pgpu_plan_s* P) { return __atomic_load_n(&P->cancel, __ATOMIC_ACQUIRE) != 0; }

// table->scans_inflight: counted from the execution's launch until its completion is seen or the plan is destroyed
void inflight_begin(pgpu_plan_s* P) {
  if (P->inflight_counted) {
    P->alone = P->table->scans_inflight.load(std::memory_order_relaxed) == 1;
    return;
  }
  P->alone = P->table->scans_inflight.fetch_add(1, std::memory_order_relaxed) == 0;
  P->inflight_counted = true;
}
void inflight_end(pgpu_plan_s* P) {
  if (!P || !P->inflight_counted || !P->table) return;
  P->table->scans_inflight.fetch_sub(1, std::memory_order_relaxed);
  P->inflight_counted = false;
}

int wait_plan(pgpu_plan_s* P, hipStream_t stream) {
  if (!P->scratch) {
    HIP_TRY(hipStreamSynchronize(stream));
    inflight_end(P);
    return 0;
  }
  Scratch* sc = P->scratch;
  if (cancelled(P)) return abandon_scratch(sc, stream) ? PGPU_ERR_DEVICE : cancel_fail();
  if (!sc->busy) HIP_TRY(hipEventCreateWithFlags(&sc->busy, hipEventDisableTiming));
  HIP_TRY(hipEventRecord(sc->busy, stream));
  // Polled, not a blocking synchronise: a pgpu_plan_cancel from another thread must end the wait.  Spinning (as the
  // HIP runtime's own synchronise does) for the first ~2 ms keeps the wake-up latency of short queries at the
  // poll interval; longer waits back off to 20 us sleeps.
  const auto t0 = std::chrono::steady_clock::now();
  // a combined plan's stream holds collectives that complete only when every peer joins them: the wait also ends at
  // the communicator's timeout, and an expired wait aborts the communicator (the collectives' kernels exit)
  int64_t comm_lim = P->comm_used ? P->comm_used->timeout_ms.load(std::memory_order_relaxed) : 0;
  if (P->comm_used && P->comm_dense && P->end_time_ms <= 0)
    comm_lim = comm_lim > 0 ? std::min(comm_lim, kDenseCombineWaitMs) : kDenseCombineWaitMs;
  for (int spin = 0;; ++spin) {
    const hipError_t e = hipEventQuery(sc->busy);
    if (e == hipSuccess) {
      inflight_end(P);
      return 0;
    }
    if (e != hipErrorNotReady) return fail(PGPU_ERR_DEVICE, "query wait failed: %s", hipGetErrorString(e));
    if (cancelled(P)) {
      sc->abandoned = true;
      if (P->comm_used) P->comm_used->abort();
      return cancel_fail();
    }
    if (P->end_time_ms > 0 && epoch_us() >= (double)P->end_time_ms * 1000.0) {
      sc->abandoned = true;
      if (P->comm_used) P->comm_used->abort();
      return timeout_fail(P);
    }
    if (comm_lim > 0 && (spin & 63) == 63 &&
        std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(comm_lim)) {
      sc->abandoned = true;
      P->comm_used->abort();
      return fail(PGPU_ERR_TIMEOUT, "the combine's collectives did not complete within the communicator's timeout "
                  "(%lld ms): a peer rank never joined them; communicator aborted", (long long)comm_lim);
    }
    if ((spin & 63) == 63 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(2))
      std::this_thread::sleep_for(std::chrono::microseconds(20));
  }
}

// Raw-value leaves of a plan: its tasks, their 256-group jobs and IN keys staged through pinned memory in one device
// buffer, then raw_leaf_bitmap_kernel writes the leaves' docbits regions (sc->docbits, sized by the caller).
int launch_raw_leaves(const pgpu_plan_s* P, Scratch* sc, hipStream_t stream) {
  if (P->raw_tasks.empty()) return 0;
  std::vector<KRawJob> jobs;
  for (size_t i = 0; i < P->raw_tasks.size(); ++i) {
    const int64_t ngroups = ((int64_t)P->raw_tasks[i].num_docs + 31) / 32;
    for (int64_t g0 = 0; g0 < ngroups; g0 += kBlock) jobs.push_back(KRawJob{(int32_t)i, (int32_t)g0});
  }
  const size_t tb = P->raw_tasks.size() * sizeof(KRawTask), jb = (jobs.size() * sizeof(KRawJob) + 15) & ~size_t(15);
  const size_t vb = std::max<size_t>(P->raw_vals.size(), 1) * 8;
  TRY(sc->rawtasks.ensure(tb + jb + vb));
  TRY(sc->rawstage.ensure(tb + jb + vb));
  uint8_t* hs = reinterpret_cast<uint8_t*>(sc->rawstage.p);
  memcpy(hs, P->raw_tasks.data(), tb);
  if (!jobs.empty()) memcpy(hs + tb, jobs.data(), jobs.size() * sizeof(KRawJob));
  if (!P->raw_vals.empty()) memcpy(hs + tb + jb, P->raw_vals.data(), P->raw_vals.size() * 8);
  HIP_TRY(hipMemcpyAsync(sc->rawtasks.p, hs, tb + jb + vb, hipMemcpyHostToDevice, stream));
  uint8_t* d = sc->rawtasks.as<uint8_t>();
  if (launch_raw_leaf_bitmaps(reinterpret_cast<const KRawJob*>(d + tb), (int64_t)jobs.size(),
                              reinterpret_cast<const KRawTask*>(d), reinterpret_cast<const int64_t*>(d + tb + jb),
                              sc->docbits.as<uint32_t>(), stream))
    return fail(PGPU_ERR_DEVICE, "raw-value filter launch failed: %s", hipGetErrorString(hipGetLastError()));
  return 0;
}

// ---- execution, in three phases so that plan_create can launch segment chunks while it still plans the rest
// (streamed plans): prologue (buffers, table init, stats), one launch per chunk of segment records, epilogue
// (star-tree kernels, slab reduce).  A plan that is not streamed is one chunk.
// KParams.pack_slot (planned with the LDS table's rows, lds_pack_slot) and narrow of a dense LDS plan, from the value
// ranges of its integer columns in every segment (sorted dictionaries: first and last entries; raw columns: their
// decoded range).  PGPU_NO_DENSE_NARROW=1: no 32-bit min / max (A/B).
void dense_lds_forms(const pgpu_plan_s* P, int32_t* pack_slot, uint32_t* narrow) {
  *pack_slot = P->mode == MODE_LDS || P->mode == MODE_HASH ? P->pack_slot : -1;  // planned with the table layout
  *narrow = 0;
  if (!P->dense || P->mode != MODE_LDS || P->num_keys <= 1 || !P->star.empty() || P->grid <= 0) return;
  for (size_t s = 0; s < P->slot_kind.size() && s < 32; ++s) {
    const int kind = P->slot_kind[s], c = P->slot_tcol[s];
    if ((kind != SLOT_MIN_KEY && kind != SLOT_MAX_KEY) || c < 0 || c == kDocIdColumn) continue;
    if (!is_int_type(P->table->types[c])) continue;
    int64_t lo = INT64_MAX, hi = INT64_MIN;
    bool known = true;
    for (const Segment* seg : P->segs) {
      const Column& col = seg->cols[c];
      if (col.raw) { lo = std::min(lo, col.raw_min); hi = std::max(hi, col.raw_max); }
      else if (!col.dict.iv.empty()) { lo = std::min(lo, col.dict.iv.front()); hi = std::max(hi, col.dict.iv.back()); }
      else if (col.dict.size() != 0) { known = false; break; }
    }
    if (!known || lo > hi || lo < 0) continue;
    if (hi < INT64_C(0xFFFFFFFF)) *narrow |= 1u << s;
  }
}

int exec_prologue(pgpu_plan_s* P, hipStream_t stream, void* d_table, int max_chunks, ExecCtx& X) {
  inflight_begin(P);
  X.t_start = trace_on() ? now_us() : 0;
  if (cancelled(P)) return cancel_fail();  // nothing is launched for a cancelled query
  uint64_t deadline = 0;
  if (P->end_time_ms > 0) {  // past the end time already: nothing is launched
    P->exec_start_ms = (int64_t)(epoch_us() / 1000.0);
    if (P->exec_start_ms >= P->end_time_ms) return timeout_fail(P);
    TRY(deadline_ticks(P->table, P->end_time_ms, &deadline));
  }
  // the state a previous execution's combine left (pgpu_plan_combine): planned slot kinds, no shard, no merged table
  if (!P->slot_kind_planned.empty()) {
    P->slot_kind = P->slot_kind_planned;
    P->slot_kind_planned.clear();
  }
  P->shard = nullptr;
  P->shard_begin = P->shard_count = 0;
  P->comm_used = nullptr;
  P->comm_dense = false;
  P->k8d_counts = false;
  P->merged_records = -1;
  Scratch* sc = P->scratch;
  X.nslots = (int)P->slot_kind.size();
  const int nslots = X.nslots;
  X.words = P->part_hash ? 0 : (int64_t)nslots * P->num_keys;  // hashed partitions: records, no table
  for (auto& e : sc->ev)
    if (!e) HIP_TRY(hipEventCreate(&e));
  if ((int)sc->cev.size() < 2 * max_chunks) {
    const size_t old = sc->cev.size();
    sc->cev.resize(2 * max_chunks, nullptr);
    for (size_t i = old; i < sc->cev.size(); ++i) HIP_TRY(hipEventCreate(&sc->cev[i]));
  }
  X.mark("events");
  PGPU_TIMING_RECORD(P, sc->ev[0], stream);
  X.mark("event 0 recorded");
  TRY(sc->sets.ensure(std::max<size_t>(std::max<size_t>(P->set_words.size(), (size_t)P->set_words_bound) * 4, 16)));
  const size_t rec_cap = std::max<size_t>((size_t)P->segs.size() * P->seg_stride, P->segrec.size());
  TRY(sc->segrec.ensure(std::max<size_t>(rec_cap, 16)));
  TRY(sc->stage.ensure(std::max<size_t>(rec_cap + (size_t)std::max<int64_t>(P->set_words_bound,
                                                                             (int64_t)P->set_words.size()) * 4, 16)));
  // Statistics words (docs matched, entries scanned, star-tree docs, timeout flag, star metric sectors): right after
  // the group table when the table is internal, so finalize reads both with one copy.  (A ring of entries zeroed 256
  // executions at a time, instead of this fill per query, was measured in r06 sessions i, j, m: no gain on C1 / C3,
  // and C4's pipelined star-tree step lost 0.17 -> 0.21 ms with the second copy it needs; not kept.)
  constexpr size_t kStatsBytes = 64;
  unsigned long long* stats;
  if (!d_table) {
    TRY(sc->table.ensure((size_t)X.words * 8 + kStatsBytes));
    stats = reinterpret_cast<unsigned long long*>(sc->table.as<uint8_t>() + (size_t)X.words * 8);
  } else {
    TRY(sc->stats.ensure(kStatsBytes));
    stats = sc->stats.as<unsigned long long>();
  }
  HIP_TRY(hipMemsetAsync(stats, 0, kStatsBytes, stream));
  P->d_stats = stats;
  P->exported = false;
  X.external = d_table != nullptr;
  X.mark("buffers");
  X.segrec = sc->segrec.as<uint8_t>();
  X.sets = sc->sets.as<uint32_t>();
  TRY(sc->tile_seg.ensure((size_t)std::max<int64_t>(std::max<int64_t>(P->num_tiles, P->tile_bound), 1) * 4));
  X.tile_seg = sc->tile_seg.as<int32_t>();
  X.from_image = P->image && P->chunks.size() == 1 && P->docbit_words == 0 && !P->set_words_bound && !P->tile_bound;
  sc->image = X.from_image ? P->image : nullptr;
  if (X.from_image) {  // build the cached plan's device image once; later executions wait for it
    DeviceImage& im = *P->image;
    std::lock_guard<std::mutex> g(im.mu);
    if (!im.uploaded) {
      const size_t rn = P->segrec.size(), sn = P->set_words.size() * 4;
      TRY(im.segrec.ensure(std::max<size_t>(rn, 16)));
      TRY(im.sets.ensure(std::max<size_t>(sn, 16)));
      TRY(im.tile_seg.ensure((size_t)std::max<int64_t>(P->num_tiles, 1) * 4));
      if (!im.built) HIP_TRY(hipEventCreateWithFlags(&im.built, hipEventDisableTiming));
      uint8_t* stage = reinterpret_cast<uint8_t*>(sc->stage.p);
      if (rn) memcpy(stage, P->segrec.data(), rn);
      for (const auto& f : P->set_fix) {
        const uint32_t* ptr = im.sets.as<uint32_t>() + f.second;
        memcpy(stage + f.first, &ptr, sizeof ptr);
      }
      if (sn) memcpy(stage + rn, P->set_words.data(), sn);
      if (rn) HIP_TRY(hipMemcpyAsync(im.segrec.p, stage, rn, hipMemcpyHostToDevice, stream));
      if (sn) HIP_TRY(hipMemcpyAsync(im.sets.p, stage + rn, sn, hipMemcpyHostToDevice, stream));
      // the plan's scan records (segments its filter prunes or its star-trees answer have none)
      const int32_t nrec = P->seg_stride > 0 ? (int32_t)(P->segrec.size() / P->seg_stride) : 0;
      if (nrec > 0 &&
          launch_expand_tiles(im.segrec.as<uint8_t>(), P->seg_stride, nrec, im.tile_seg.as<int32_t>(), 0,
                              stats, stream))
        return fail(PGPU_ERR_DEVICE, "expand launch failed: %s", hipGetErrorString(hipGetLastError()));
      HIP_TRY(hipEventRecord(im.built, stream));
      im.uploaded = true;
    } else if (!im.ready) {
      if (hipEventQuery(im.built) == hipSuccess) im.ready = true;
      else HIP_TRY(hipStreamWaitEvent(stream, im.built, 0));
    }
    X.segrec = im.segrec.as<uint8_t>();
    X.sets = im.sets.as<uint32_t>();
    X.tile_seg = im.tile_seg.as<int32_t>();
  }
  X.mark("image");
  if (P->docbit_words > 0) TRY(sc->docbits.ensure((size_t)P->docbit_words * 4));
  if (!P->bit_blocks.empty()) {  // BitmapBasedFilterOperator leaves: OR the matching dictIds' containers
    TRY(sc->bittasks.ensure(std::max<size_t>(P->bit_tasks.size(), 1) * sizeof(KBitTask)));
    TRY(sc->bitblocks.ensure(P->bit_blocks.size() * sizeof(KBitBlock)));
    // staged through pinned memory: asynchronous copies (pageable sources would block the host)
    const size_t tb = P->bit_tasks.size() * sizeof(KBitTask), bb = P->bit_blocks.size() * sizeof(KBitBlock);
    TRY(sc->bitstage.ensure(tb + bb));
    uint8_t* hs = reinterpret_cast<uint8_t*>(sc->bitstage.p);
    if (tb) memcpy(hs, P->bit_tasks.data(), tb);
    memcpy(hs + tb, P->bit_blocks.data(), bb);
    if (tb) HIP_TRY(hipMemcpyAsync(sc->bittasks.p, hs, tb, hipMemcpyHostToDevice, stream));
    HIP_TRY(hipMemcpyAsync(sc->bitblocks.p, hs + tb, bb, hipMemcpyHostToDevice, stream));
    if (launch_inv_materialize(sc->bitblocks.as<KBitBlock>(), (int64_t)P->bit_blocks.size(),
                               sc->bittasks.as<KBitTask>(), sc->docbits.as<uint32_t>(), stream))
      return fail(PGPU_ERR_DEVICE, "inverted-index materialise launch failed: %s",
                  hipGetErrorString(hipGetLastError()));
  }
  TRY(launch_raw_leaves(P, sc, stream));  // raw-value leaves' docbits regions
  uint64_t* table = d_table ? reinterpret_cast<uint64_t*>(d_table) : sc->table.as<uint64_t>();
  X.table = table;
  P->d_table_used = table;
  KParams& kp = X.kp;
  memset(&kp, 0, sizeof kp);
  kp.pack_slot = -1;
  kp.deadline = deadline;
  kp.seg_stride = P->seg_stride;
  kp.num_cols = (int)P->query_cols.size();
  kp.num_ops = (int)P->ops.size();
  kp.pure_and = P->pure_and ? 1 : 0;
  for (size_t i = 0; i < P->ops.size(); ++i) kp.ops[i] = P->ops[i];
  kp.num_leaves = P->num_leaves;
  for (int i = 0; i < P->num_leaves; ++i) kp.leaf_col[i] = P->leaf_slot[i];
  kp.num_keys = (int)P->key_cols.size();
  for (size_t j = 0; j < P->key_cols.size(); ++j) {
    int slot = 0;
    for (size_t i = 0; i < P->query_cols.size(); ++i) if (P->query_cols[i] == P->key_cols[j]) slot = (int)i;
    kp.key_col[j] = slot;
    kp.key_stride[j] = P->key_stride[j];
  }
  kp.num_keys_total = P->num_keys;
  kp.key_bias = P->key_bias;
  kp.tile_shift = P->tile_shift;
  // Tile order: interleaved (the tiles in flight on an XCD come from ~one segment: its dictionaries stay in that
  // XCD's L2 for the per-doc gathers) or chunked (a workgroup's tiles follow each other in one segment: its records
  // and leaf registers are loaded once per run).  Plans with many matches (dense, and the sparse ones of estimated
  // selectivity >= 1/16) gather enough to want the former: C4's scan path 151 -> 141 us interleaved, where C3
  // (0.18 %) loses 7 % and the indexed C3 15 % (profiles/r05_ab_summary.txt, session za).
#ifdef PGPU_CHUNK_ALL  // (an A/B build of the library: contiguous runs for the dense and wide plans too)
  kp.tile_chunks = 1;
#else
  kp.tile_chunks = P->dense || P->fast_wide ? 0 : 1;
#endif
  kp.num_slots = nslots;
  for (int sl = 0; sl < nslots; ++sl) { kp.slot_kind[sl] = P->slot_kind[sl]; kp.slot_col[sl] = P->slot_col[sl]; }
  kp.pair_leaves = 1;
  dense_lds_forms(P, &kp.pack_slot, &kp.narrow);
  kp.pack_shift = P->pack_shift;
  kp.stats = stats;
  if (P->leap_reserved) {  // one byte per (tile, wave) of the plan, written by the scan kernel for LEAP2 segments
    TRY(sc->leap_maps.ensure((size_t)std::max<int64_t>(std::max<int64_t>(P->num_tiles, P->tile_bound), 1) *
                             (kBlock / 64)));
    kp.leap_maps = sc->leap_maps.as<uint8_t>();
  }
  const int star_blocks = P->star_batches * P->star_chunks;
  if (P->mode == MODE_LDS) {
    TRY(sc->slab.ensure((size_t)std::max(max_chunks * P->grid + star_blocks, 1) * X.words * 8));
    kp.slab = sc->slab.as<uint64_t>();
  } else {
    if (P->mode == MODE_HASH && !P->part_hash) {
      TRY(sc->hash_keys.ensure((size_t)P->num_keys * 8));
      kp.hash_keys = sc->hash_keys.as<unsigned long long>();
      if (!P->stage_end.empty()) {
        int64_t total = 0;
        kp.num_stages = (int)P->stage_end.size();
        for (int s = 0; s < kp.num_stages; ++s) {
          kp.stage_end[s] = P->stage_end[s];
          kp.stage_cap[s] = P->stage_cap[s];
          kp.stage_mult[s] = P->stage_mult[s];
          kp.stage_off[s] = total;
          total += P->stage_cap[s];
        }
        TRY(sc->stage_keys.ensure((size_t)total * 8));
        HIP_TRY(hipMemsetAsync(sc->stage_keys.p, 0xFF, (size_t)total * 8, stream));  // every slot empty (~0)
        kp.stage_keys = sc->stage_keys.as<unsigned long long>();
      }
    }
    if (!P->partitioned &&  // the partitioned path stores every table word itself
        launch_table_init(table, P->slot_kind.data(), nslots, P->num_keys, kp.hash_keys, stream))
      return fail(PGPU_ERR_DEVICE, "table init launch failed: %s", hipGetErrorString(hipGetLastError()));
    kp.table = table;
  }
  P->launches_done = 0;
  return 0;
}

// Uploads chunk c's records (SET pointers patched to the device bitsets) and its bitset words.
int exec_upload_chunk(pgpu_plan_s* P, hipStream_t stream, const ExecCtx& X, const LaunchChunk& C) {
  if (X.from_image) return 0;  // the cached plan's device image holds the records
  Scratch* sc = P->scratch;
  uint8_t* stage = reinterpret_cast<uint8_t*>(sc->stage.p);
  const size_t r0 = (size_t)C.rec_begin * P->seg_stride, rn = (size_t)C.num_recs * P->seg_stride;
  if (rn) memcpy(stage + r0, P->segrec.data() + r0, rn);
  for (int64_t i = C.fix_begin; i < C.fix_end; ++i) {
    const auto& f = P->set_fix[i];
    const uint32_t* ptr = sc->sets.as<uint32_t>() + f.second;
    memcpy(stage + f.first, &ptr, sizeof ptr);
  }
  for (const auto& f : P->bit_fix)
    if (f.first >= (int64_t)r0 && f.first < (int64_t)(r0 + rn)) {
      const uint32_t* ptr = sc->docbits.as<uint32_t>() + f.second;
      memcpy(stage + f.first, &ptr, sizeof ptr);
    }
  if (rn) HIP_TRY(hipMemcpyAsync(sc->segrec.as<uint8_t>() + r0, stage + r0, rn, hipMemcpyHostToDevice, stream));
  if (C.set_end > C.set_begin) {
    const size_t set_off = (size_t)P->segs.size() * P->seg_stride + (size_t)C.set_begin * 4;
    const size_t bytes = (size_t)(C.set_end - C.set_begin) * 4;
    if (set_off + bytes > sc->stage.cap) return fail(PGPU_ERR_DEVICE, "set staging overflow");
    memcpy(stage + set_off, P->set_words.data() + C.set_begin, bytes);
    HIP_TRY(hipMemcpyAsync(sc->sets.as<uint32_t>() + C.set_begin, stage + set_off, bytes, hipMemcpyHostToDevice,
                           stream));
  }
  return 0;
}

// Launches the scan of chunk c (records already uploaded): tile map of its records, then the scan kernel (or the
// partitioned group-by) over its tiles into slab region c.
// PGPU_TRACE=check (diagnostics): before a scan launch, the records and tile map the kernel will read are copied
// back and compared with the plan's host records (pointer fields patched at upload skipped); a mismatch fails the
// query (PGPU_ERR_DEVICE) instead of launching on them.
bool check_launch_on() {
  static const bool on = diag("check");
  return on;
}
int check_launch_inputs(const pgpu_plan_s* P, hipStream_t stream, const ExecCtx& X, const LaunchChunk& C) {
  HIP_TRY(hipStreamSynchronize(stream));
  const size_t r0 = (size_t)C.rec_begin * P->seg_stride, rn = (size_t)C.num_recs * P->seg_stride;
  std::vector<uint8_t> dev(rn);
  std::vector<int32_t> tiles((size_t)std::max<int64_t>(C.num_tiles, 0));
  if (rn) HIP_TRY(hipMemcpy(dev.data(), X.segrec + r0, rn, hipMemcpyDeviceToHost));
  if (!tiles.empty()) HIP_TRY(hipMemcpy(tiles.data(), X.tile_seg + C.tile_begin, tiles.size() * 4, hipMemcpyDeviceToHost));
  if (P->segrec.size() >= r0 + rn) {
    std::vector<char> skip(rn, 0);
    auto mark = [&](int64_t off) {
      if (off >= (int64_t)r0 && off + 8 <= (int64_t)(r0 + rn)) memset(skip.data() + (off - r0), 1, 8);
    };
    for (const auto& f : P->set_fix) mark(f.first);
    for (const auto& f : P->bit_fix) mark(f.first);
    for (size_t i = 0; i < rn; ++i)
      if (!skip[i] && dev[i] != P->segrec[r0 + i])
        return fail(PGPU_ERR_DEVICE, "launch check: device record byte %zu differs from the plan (%u vs %u)", r0 + i,
                    dev[i], P->segrec[r0 + i]);
  }
  int32_t prev = 0;
  for (size_t i = 0; i < tiles.size(); ++i) {
    if (tiles[i] < prev || tiles[i] >= C.num_recs)
      return fail(PGPU_ERR_DEVICE, "launch check: tile %zu maps to record %d of %lld", i, tiles[i],
                  (long long)C.num_recs);
    prev = tiles[i];
  }
  return 0;
}

// The scan instance a plan launches (k_direct.hip): 2 dense "simple", 1 dense, 3 index + scan pair, 5 / 4 pure-AND
// sparse with 4 / 2-doc lane batches, 0 the general sparse one.
int scan_variant(const pgpu_plan_s* P) {
  return P->dense_simple ? 2 : P->dense ? 1 : P->pair_variant ? 3 : P->fast_wide ? 5 : P->fast_variant ? 4 : 0;
}

// PGPU_TRACE=wgtimes with a PGPU_DIAG_WG_TIMES build: every scan launch is synchronised and its workgroups' start /
// tile-loop end / end times (wall clock, relative to the earliest start) summarised on stderr -- how much of a launch
// is its ramp, its tail and the imbalance of the static tile split.
unsigned long long* g_diag_times = nullptr;
int diag_wg_times_begin(KParams& kp, int grid, hipStream_t stream) {
  constexpr int kMaxWgs = 1 << 16;
  if (grid > kMaxWgs) return 0;
  if (!g_diag_times) HIP_TRY(hipMalloc(&g_diag_times, (size_t)kMaxWgs * 64));
  HIP_TRY(hipMemsetAsync(g_diag_times, 0, (size_t)grid * 64, stream));
  kp.diag_times = g_diag_times;
  return 0;
}

int diag_wg_times_report(pgpu_table_s* t, const KParams& kp, int grid, hipStream_t stream) {
  if (!kp.diag_times) return 0;
  std::vector<unsigned long long> h((size_t)grid * 8);
  HIP_TRY(hipMemcpyAsync(h.data(), kp.diag_times, h.size() * 8, hipMemcpyDeviceToHost, stream));
  HIP_TRY(hipStreamSynchronize(stream));
  int khz = 100000;
  hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, t->device);
  const double us = 1000.0 / khz;
  unsigned long long t0 = ~0ull;
  for (int b = 0; b < grid; ++b) if (h[8 * b + 2]) t0 = std::min(t0, h[8 * b]);
  if (t0 == ~0ull) return 0;
  std::vector<double> st, le, en, tiles;
  double xcd_end[8] = {0};
  // PGPU_WGTIMES_OUT=<file>: every workgroup's raw row appended (launch separator "# grid tiles")
  FILE* raw = getenv("PGPU_WGTIMES_OUT") ? fopen(getenv("PGPU_WGTIMES_OUT"), "a") : nullptr;
  if (raw) fprintf(raw, "# %d %lld\n", grid, (long long)kp.num_tiles);
  for (int b = 0; b < grid; ++b) {
    const unsigned long long* d = &h[8 * (size_t)b];
    if (!d[2]) continue;
    st.push_back((d[0] - t0) * us);
    le.push_back((d[1] - t0) * us);
    en.push_back((d[2] - t0) * us);
    tiles.push_back((double)(d[3] & 0xffffffffu));
    xcd_end[d[5] & 7] = std::max(xcd_end[d[5] & 7], en.back());
    if (raw)
      fprintf(raw, "%d %.2f %.2f %.2f %llu %llu %llu %llu\n", b, st.back(), le.back(), en.back(), d[3] & 0xffffffffu,
              d[3] >> 32, d[4], d[5]);
  }
  if (raw) fclose(raw);
  auto pct = [](std::vector<double> v, double q) {
    std::sort(v.begin(), v.end());
    return v[std::min(v.size() - 1, (size_t)(q * (v.size() - 1) + 0.5))];
  };
  fprintf(stderr, "[pgpu] wgtimes grid %d tiles %d: start p50 %.1f max %.1f | loop end p0 %.1f p10 %.1f p50 %.1f p90 %.1f "
          "max %.1f | end max %.1f us | tiles/wg %.0f..%.0f | xcd end %.1f %.1f %.1f %.1f %.1f %.1f %.1f %.1f\n",
          grid, kp.num_tiles, pct(st, 0.5), pct(st, 1.0), pct(le, 0.0), pct(le, 0.1), pct(le, 0.5), pct(le, 0.9),
          pct(le, 1.0), pct(en, 1.0), pct(tiles, 0.0), pct(tiles, 1.0), xcd_end[0], xcd_end[1], xcd_end[2], xcd_end[3],
          xcd_end[4], xcd_end[5], xcd_end[6], xcd_end[7]);
  return 0;
}

// Run-time claims of a chunked scan launch (KParams.claim; library builds with -DPGPU_TILE_CLAIMS only): the static
// runs cover the first PGPU_CLAIM_STATIC_PM / 1000 of the tiles and the rest is claimed in runs of 1/PGPU_CLAIM_DIV
// of a workgroup's share.  The counters are u32 words 12..15 of the statistics block (zeroed per execution): launches
// 0-3 of a plan.  Measured on MI355X and not the default (r06 session b, profiles/r06_ab_summary.txt): C3's scan
// 729 -> 711 us at 1000 segments but its pipelined step 0.687 -> 0.719 ms, and at 125 segments 119 -> 145 us (every
// claimed tile reloads its segment's records behind a workgroup barrier).
#ifndef PGPU_CLAIM_STATIC_PM
#define PGPU_CLAIM_STATIC_PM 750
#endif
#ifndef PGPU_CLAIM_DIV
#define PGPU_CLAIM_DIV 16
#endif
// Chunked scans: each workgroup's run of tiles weighted by the CU slot it is dispatched to (KParams.slot_w), for a
// launch that has the CUs to itself (P->alone: its workgroups' slots are their dispatch order; beside another query's
// scan the freed slots go to the newcomers in no such order) and >= kSlotWeightMinShare tiles per workgroup.  The SIMDs
// issue the oldest wave first: equal shares end slot by slot, 1 : 1.08 : 1.17 : 1.27 (C3, 125 and 1000 segments), and
// weighted by those ratios the per-tile times spread further (4.55 / 4.92 / 5.47 / 6.06 us at 1000 segments), so
// pgpu_config.slot_weight_step defaults to the latter's inverse, 1 + 0.11 (S-1-s) (r06 sessions f, g:
// profiles/r06_ab_summary.txt); 0 gives equal shares.
constexpr int64_t kSlotWeightMinShare = 32;
void set_slot_weights(KParams& kp, int grid, int num_cus, double step) {
  kp.slot_n = 0;
  const int S = num_cus > 0 && grid % num_cus == 0 ? grid / num_cus : 0;
  if (!(step > 0.0) || !kp.tile_chunks || S < 2 || S > 4 || (grid & 7) || kp.claim ||
      kp.num_tiles < kSlotWeightMinShare * grid)
    return;
  for (int s = 0; s < S; ++s) kp.slot_w[s] = (uint16_t)std::min(4096.0, (1.0 + step * (S - 1 - s)) * 256.0 + 0.5);
  kp.slot_n = S;
}

void set_tile_claims(KParams& kp, unsigned long long* d_stats, int grid, int launch) {
  kp.claim = nullptr;
#ifdef PGPU_TILE_CLAIMS
  const int64_t share = (int64_t)kp.num_tiles / std::max(grid, 1);
  if (!kp.tile_chunks || grid < 64 || (grid & 7) || launch >= 4 || share < 8) return;
  kp.claim = reinterpret_cast<unsigned int*>(d_stats + 6) + launch;
  kp.claim_base = (int32_t)((int64_t)kp.num_tiles * PGPU_CLAIM_STATIC_PM / 1000);
  kp.claim_tiles = (int32_t)std::max<int64_t>(1, share / PGPU_CLAIM_DIV);
#endif
}

int exec_launch_chunk(pgpu_plan_s* P, hipStream_t stream, ExecCtx& X, const LaunchChunk& C, int c) {
  Scratch* sc = P->scratch;
  KParams kp = X.kp;
  kp.segs = X.segrec + (size_t)C.rec_begin * P->seg_stride;
  kp.num_segs = (int)C.num_recs;
  kp.num_tiles = (int32_t)C.num_tiles;
  kp.tile_seg = X.tile_seg + C.tile_begin;
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(P->grid, C.num_tiles));
  if (P->mode == MODE_LDS) kp.slab = X.kp.slab + X.slabs_used * X.words;
  if (kp.leap_maps) kp.leap_maps += C.tile_begin * (kBlock / 64);
  if (X.from_image) {  // the tile map is in the image; only the deadline gate remains (and only with a deadline)
    if (C.num_tiles > 0 && kp.deadline && launch_deadline_gate(kp.deadline, kp.stats, stream))
      return fail(PGPU_ERR_DEVICE, "gate launch failed: %s", hipGetErrorString(hipGetLastError()));
  } else if (C.num_recs > 0 && launch_expand_tiles(kp.segs, kp.seg_stride, kp.num_segs, X.tile_seg + C.tile_begin,
                                                   kp.deadline, kp.stats, stream)) {
    return fail(PGPU_ERR_DEVICE, "expand launch failed: %s", hipGetErrorString(hipGetLastError()));
  }
  if (check_launch_on()) TRY(check_launch_inputs(P, stream, X, C));
  X.mark("chunk set up");
  if (c == 0) PGPU_TIMING_RECORD(P, sc->ev[1], stream);
  PGPU_TIMING_RECORD(P, sc->cev[2 * c], stream);
  if (C.num_tiles > 0 && P->partitioned) {
    const int nslots = X.nslots;
    KPartParams pp;
    memset(&pp, 0, sizeof pp);
    pp.base = kp;
    pp.pshift = P->part_shift;
    pp.num_parts = P->num_parts;
    pp.num_streams = (int)P->stream_col.size();
    for (size_t j = 0; j < P->stream_col.size(); ++j) { pp.stream_col[j] = P->stream_col[j]; pp.stream_f64[j] = P->stream_f64[j]; }
    for (int sl = 0; sl < nslots; ++sl) pp.slot_stream[sl] = P->slot_stream[sl];
    const int64_t cap = std::max<int64_t>(P->total_docs, 1);
    TRY(sc->part_start.ensure((size_t)(P->num_parts + 1) * 4));
    const int cshift = part_coarse_shift(P->num_parts);
    pp.cshift = cshift;
    pp.num_coarse = part_coarse_runs(P->num_parts);
    pp.chunks_per_coarse = std::max(1, 1024 / pp.num_coarse);
    {  // K8e batch: as many records as fit 96 KB of LDS beside the per-partition counters, a multiple of kBlock
      const int kb = P->part_hash ? 4 : 2;  // staged key bytes
      const int64_t fixed = (int64_t)part_split_lds(cshift, pp.num_streams, 0, kb);
      const int64_t b = (96 * 1024 - fixed) / (8 * pp.num_streams + 4 + kb) / kBlock * kBlock;
      pp.split_batch = (int)std::max<int64_t>(kBlock, std::min<int64_t>(kSplitBatch, b));
    }
    TRY(sc->coarse_fill.ensure((size_t)pp.num_coarse * 4));
    TRY(sc->fine_fill.ensure((size_t)P->num_parts * 4));
    if (cshift > 0) {
      TRY(sc->mid_key.ensure((size_t)cap * 4));
      TRY(sc->mid_val.ensure(std::max<size_t>((size_t)cap * 8 * pp.num_streams, 8)));
      pp.mid_key = sc->mid_key.as<uint32_t>();
      pp.mid_val = sc->mid_val.as<uint64_t>();
    }
    pp.coarse_fill = sc->coarse_fill.as<uint32_t>();
    pp.fine_fill = sc->fine_fill.as<uint32_t>();
    if (P->part_hash) {
      pp.hashed = 1;
      pp.mid_pair = cshift > 0 && pp.num_streams == 1 && P->part_val32 && !P->stream_f64[0] ? 1 : 0;
      pp.pbits = P->part_pbits;
      pp.sbits = P->part_sbits;
      TRY(sc->rec_key32.ensure((size_t)cap * 4));
      pp.rec_key32 = sc->rec_key32.as<uint32_t>();
      // the groups' compacted records, where finalize's compaction of a hash table would put them
      const int64_t ocap = part_hash_out_cap(P);
      TRY(sc->ckeys.ensure((size_t)ocap * 8 * (1 + nslots)));
      TRY(sc->counter.ensure(64));
      HIP_TRY(hipMemsetAsync(sc->counter.p, 0, 8, stream));
      pp.out_rec = sc->ckeys.as<uint64_t>();
      pp.out_count = sc->counter.as<unsigned long long>();
      pp.out_cap = ocap;
      TRY(sc->part_mm.ensure((size_t)P->num_parts * 2 * nslots * 8));
      pp.out_mm = sc->part_mm.as<unsigned long long>();
      P->part_hash_live = true;
    } else {
      TRY(sc->rec_key.ensure((size_t)cap * 2));
    }
    TRY(sc->rec_val.ensure(std::max<size_t>((size_t)cap * 8 * pp.num_streams, 8)));
    pp.part_start = sc->part_start.as<uint32_t>();
    pp.rec_key = sc->rec_key.as<uint16_t>();
    pp.rec_val = sc->rec_val.as<uint64_t>();
    pp.rec_cap = cap;
    pp.val32 = P->part_val32 ? 1 : 0;
    if (P->part_hash && P->part_pack_range >= 0 && pp.num_streams == 1 && pp.val32 && P->part_pbits >= 1) {
      // hashed partitions: K8e's records packed as hk below the partition bits | (value - pack_min) above them
      int vb = 0;
      while (vb < 32 && (P->part_pack_range >> vb) != 0) ++vb;
      if (vb <= P->part_pbits) {
        pp.fine_pack = 1;
        pp.pack_min = P->part_pack_min;
        pp.pack_range = P->part_pack_range;
        pp.cs_pack = nslots == 2 && P->slot_kind[0] == SLOT_COUNT && P->slot_kind[1] == SLOT_SUM_I64 &&
                     P->slot_stream[1] == 0 ? 1 : 0;
      }
    } else if (!P->part_hash && cshift > 0 && P->part_pack_range >= 0) {
      const int free_bits = 32 - (pp.pshift + cshift);
      int vb = 0;
      while (vb < free_bits && (P->part_pack_range >> vb) != 0) ++vb;
      if ((P->part_pack_range >> vb) == 0) {
        pp.pack_bits = std::max(vb, 1);
        pp.pack_min = P->part_pack_min;
        pp.fine_pack = pp.pshift + pp.pack_bits <= 32 && pp.num_streams == 1 ? 1 : 0;
        pp.cs_pack = pp.fine_pack && nslots == 2 && P->slot_kind[0] == SLOT_COUNT &&
                     P->slot_kind[1] == SLOT_SUM_I64 && P->slot_stream[1] == 0 ? 1 : 0;
        pp.pack_range = P->part_pack_range;
      }
    }
    int grid = P->part_grid;
#ifndef PGPU_PART_NO_STAGE  // (defined only by an A/B build of the library: every record stored from its lane)
    // one-word records with <= 64 coarse runs: K8c stages each wave's records by run in LDS and stores them in runs;
    // the grid (K8a's too) follows that instance's occupancy
    pp.staged = pp.cshift > 0 && pp.num_coarse <= 64 ? (pp.pack_bits > 0 ? 1 : pp.mid_pair ? 2 : 0) : 0;
    if (pp.staged) {
      if (P->part_grid_staged[pp.staged - 1] <= 0) {
        const int per_cu =
            std::max(1, std::min(occupancy_part_pass(P->part_lds, P->num_parts, pp.num_coarse, pp.staged), 4));
        P->part_grid_staged[pp.staged - 1] =
            (int)std::max<int64_t>(1, std::min<int64_t>(P->num_tiles, (int64_t)P->table->num_cus * per_cu));
      }
      grid = P->part_grid_staged[pp.staged - 1];
    }
#endif
    TRY(sc->block_off.ensure((size_t)grid * pp.num_coarse * 4));
    pp.block_off = sc->block_off.as<uint32_t>();
    // K8d's partitions are the ordered compaction's chunks (C5): K8d writes their counts and ranges, and finalize
    // skips compact_count_kernel's pass over the table (P->k8d_counts)
    {
      const int64_t G = P->num_keys, nch = compact_ordered_chunks(G);
      if (pp.cs_pack && !P->hash && ((int64_t)1 << pp.pshift) == kCompactChunkKeys && nch == P->num_parts &&
          (int64_t)nslots * G * 8 > kHostCompactBytes) {
        TRY(sc->cslots.ensure(compact_scratch_bytes(G, nslots)));
        pp.chunk_cnt = sc->cslots.as<uint32_t>();
        pp.chunk_mm = reinterpret_cast<long long*>(sc->cslots.as<uint8_t>() + ((nch * 4 + 7) & ~int64_t(7)));
        P->k8d_counts = true;
      }
    }
    if (launch_partitioned(pp, grid, P->part_lds, stream))
      return fail(PGPU_ERR_DEVICE, "partitioned group-by launch failed: %s", hipGetErrorString(hipGetLastError()));
  } else if (C.num_tiles > 0) {
    static const bool wg_times = diag("wgtimes");
    if (wg_times) TRY(diag_wg_times_begin(kp, grid, stream));
    set_tile_claims(kp, P->d_stats, grid, c);
    if (P->alone) set_slot_weights(kp, grid, P->table->num_cus, P->cfg.slot_weight_step);
    const int rc = launch_filter_groupby(kp, P->mode,
                                         scan_variant(P),
                                         grid, P->lds_bytes, stream);
    if (rc) return fail(PGPU_ERR_DEVICE, "scan launch failed: %s", hipGetErrorString(hipGetLastError()));
    X.mark("scan launched");
    if (wg_times) TRY(diag_wg_times_report(P->table, kp, grid, stream));
  }
  PGPU_TIMING_RECORD(P, sc->cev[2 * c + 1], stream);
  if (C.num_tiles > 0 && P->any_leap2 && P->leap_reserved && !P->partitioned) {
    if (P->chunks.size() == 1 && P->mode == MODE_LDS) {  // folded into the epilogue's launch
      X.leap_segs = kp.segs;
      X.leap_nsegs = kp.num_segs;
    } else if (launch_leap2_compose(kp.segs, kp.seg_stride, kp.num_segs, kp.leap_maps, kp.stats, stream)) {
      return fail(PGPU_ERR_DEVICE, "filter statistics launch failed: %s", hipGetErrorString(hipGetLastError()));
    }
  }
  if (C.num_tiles > 0 && !P->partitioned && P->mode == MODE_LDS) X.slabs_used += grid;
  P->launches_done = c + 1;
  return 0;
}

int exec_epilogue(pgpu_plan_s* P, hipStream_t stream, ExecCtx& X) {
  Scratch* sc = P->scratch;
  const int nslots = X.nslots;
  const int64_t words = X.words;
  KParams& kp = X.kp;
  const int nl = P->launches_done;
  if (nl == 0) PGPU_TIMING_RECORD(P, sc->ev[1], stream);
  if (!P->star.empty()) {
    // star-tree segments: K5 traversal then K6 residual scan + aggregation into the same group table
    X.mark("before star buffers");
    TRY(sc->starwork.ensure((size_t)P->star_work_bytes + P->star.size() * 8 + 16));
    int64_t* seg_total = reinterpret_cast<int64_t*>(sc->starwork.as<uint8_t>() + P->star_work_bytes);
    {
      const void* before = sc->starrec.p;
      TRY(sc->starrec.ensure(P->star.size() * sizeof(KStarSeg)));
      if (sc->starrec.p != before) sc->starrec_sent.clear();  // a new buffer holds nothing yet
    }
    std::vector<KStarSeg> recs = P->star;
    for (size_t i = 0; i < recs.size(); ++i) {
      uint8_t* base = sc->starwork.as<uint8_t>() + P->star_work_off[i];
      const int64_t nn = recs[i].num_nodes;
      recs[i].ranges = reinterpret_cast<int32_t*>(base);
      recs[i].prefix = reinterpret_cast<int64_t*>(base + ((2 * nn * 4 + 7) & ~int64_t(7)));
      recs[i].frontier = reinterpret_cast<int32_t*>(base + ((2 * nn * 4 + 7) & ~int64_t(7)) + (nn + 1) * 8);
      recs[i].out = recs[i].frontier + 6 * nn;
    }
    for (auto& f : P->star_match_fix)
      recs[std::get<0>(f)].match[std::get<1>(f)] = X.sets + std::get<2>(f);
    // The records (this scratch's work buffers, the plan's match sets) are the same for every execution of a cached
    // plan on this scratch: uploaded when they differ from the last upload.  A small host-to-device copy could block
    // the host for milliseconds behind other streams' work (C4 at 3 queries in flight: 5.4 ms in one execution).
    const size_t rbytes = recs.size() * sizeof(KStarSeg);
    X.mark("star buffers + records built");
    if (sc->starrec_sent.size() != rbytes || memcmp(sc->starrec_sent.data(), recs.data(), rbytes) != 0) {
      TRY(sc->starstage.ensure(rbytes));
      memcpy(sc->starstage.p, recs.data(), rbytes);
      HIP_TRY(hipMemcpyAsync(sc->starrec.p, sc->starstage.p, rbytes, hipMemcpyHostToDevice, stream));
      sc->starrec_sent.assign(reinterpret_cast<const uint8_t*>(recs.data()),
                              reinterpret_cast<const uint8_t*>(recs.data()) + rbytes);
    }
    X.mark("star records copy queued");
    if (launch_startree_traverse(sc->starrec.as<KStarSeg>(), (int)recs.size(), seg_total, kp.deadline, kp.stats,
                                 stream))
      return fail(PGPU_ERR_DEVICE, "star-tree traversal launch failed: %s", hipGetErrorString(hipGetLastError()));
    X.mark("K5 launched");
    KStarParams sp;
    memset(&sp, 0, sizeof sp);
    sp.num_wgs = P->star_chunks;
    sp.range_cache = P->star_range_cache;
    sp.num_keys = (int)P->key_cols.size();
    for (size_t j = 0; j < P->key_cols.size(); ++j) sp.key_stride[j] = P->key_stride[j];
    sp.key_bias = P->key_bias;
    sp.num_keys_total = P->num_keys;
    sp.num_slots = nslots;
    for (int sl = 0; sl < nslots; ++sl) {
      sp.slot_kind[sl] = P->slot_kind[sl];
      sp.slot_int[sl] = sl > 0 && P->slot_tcol[sl] >= 0 && is_int_type(P->table->types[P->slot_tcol[sl]]) ? 1 : 0;
    }
    sp.table = kp.table;
    sp.slab = P->mode == MODE_LDS ? kp.slab + X.slabs_used * words : nullptr;
    sp.hash_keys = kp.hash_keys;
    sp.stats = kp.stats;
    sp.deadline = kp.deadline;
    sp.cache_ints = P->star_cache_ints;
    for (int b = 0; b < P->star_batches; ++b) {  // kStarMaxSegs segments per launch, slabs back to back
      const int s0 = b * kStarMaxSegs;
      sp.segs = sc->starrec.as<KStarSeg>() + s0;
      sp.num_segs = (int)std::min<int64_t>(kStarMaxSegs, (int64_t)recs.size() - s0);
      sp.seg_total = seg_total + s0;
      if (P->mode == MODE_LDS) sp.slab = kp.slab + (X.slabs_used + (int64_t)b * P->star_chunks) * words;
      if (launch_startree_scan(sp, P->mode, P->star_lds_bytes, stream))
        return fail(PGPU_ERR_DEVICE, "star-tree scan launch failed: %s", hipGetErrorString(hipGetLastError()));
      X.mark("K6 launched");
    }
  }
  if (!P->generic.empty()) {
    // STATS_GENERIC segments: the leaves' match bitmaps, read back and replayed on the host at finalize
    std::vector<KMaskJob> jobs;
    for (const auto& g : P->generic)
      for (int64_t g0 = 0; g0 < ((int64_t)g.num_docs + 31) / 32; g0 += kBlock)
        jobs.push_back(KMaskJob{(int32_t)g.rec, (int32_t)g0, g.out_word});
    TRY(sc->mask_jobs.ensure(std::max<size_t>(jobs.size(), 1) * sizeof(KMaskJob)));
    TRY(sc->leaf_masks.ensure((size_t)std::max<int64_t>(P->generic_words, 1) * 4));
    TRY(sc->maskstage.ensure(std::max<size_t>(jobs.size() * sizeof(KMaskJob), (size_t)P->generic_words * 4) + 16));
    memcpy(sc->maskstage.p, jobs.data(), jobs.size() * sizeof(KMaskJob));
    HIP_TRY(hipMemcpyAsync(sc->mask_jobs.p, sc->maskstage.p, jobs.size() * sizeof(KMaskJob), hipMemcpyHostToDevice,
                           stream));
    KParams mp = kp;
    mp.segs = X.segrec;
    if (launch_leaf_masks(mp, sc->mask_jobs.as<KMaskJob>(), (int32_t)jobs.size(), sc->leaf_masks.as<uint32_t>(),
                          stream))
      return fail(PGPU_ERR_DEVICE, "leaf mask launch failed: %s", hipGetErrorString(hipGetLastError()));
    HIP_TRY(hipMemcpyAsync(sc->maskstage.p, sc->leaf_masks.p, (size_t)P->generic_words * 4, hipMemcpyDeviceToHost,
                           stream));
  }
  PGPU_TIMING_RECORD(P, sc->ev[2], stream);
  X.mark("event 2 recorded");
  if (P->mode == MODE_LDS) {
    // fold every slab written: the scan launches' (back to back) and the star-tree chunks' after them
    const int64_t all = X.slabs_used + (int64_t)P->star_batches * P->star_chunks;
    if (all == 0) {
      if (launch_table_init(X.table, P->slot_kind.data(), nslots, P->num_keys, nullptr, stream))
        return fail(PGPU_ERR_DEVICE, "table init launch failed");
    } else {
      // PGPU_EPILOGUE_EXPORT (an A/B build of the library only): for small internal tables the epilogue's last block
      // also writes table + statistics to pinned host memory and finalize launches no copy.  Measured and not the
      // default (r06 sessions i, j): the copy launch goes, but the host sees the stream complete ~10-15 us later
      // (C1 latency 0.057 -> 0.071 ms, C3 at 125 segments 0.163 -> 0.169).
#ifdef PGPU_EPILOGUE_EXPORT
      const bool exp = !X.external && X.words * 8 <= kExportBytes;
#else
      const bool exp = false;
#endif
      if (exp) {
        TRY(sc->exported.ensure((size_t)X.words * 8 + 64));
        if (!sc->export_done.p) {
          TRY(sc->export_done.ensure(64));
          HIP_TRY(hipMemsetAsync(sc->export_done.p, 0, 64, stream));
        }
      }
      if (launch_epilogue(kp.slab, P->slot_kind.data(), nslots, P->num_keys, (int32_t)all, X.table, X.leap_segs,
                          P->seg_stride, X.leap_nsegs, kp.leap_maps, kp.stats,
                          exp ? reinterpret_cast<uint64_t*>(sc->exported.p) : nullptr, exp ? sc->export_done.as<unsigned int>() : nullptr,
                          stream))
        return fail(PGPU_ERR_DEVICE, "reduce launch failed: %s", hipGetErrorString(hipGetLastError()));
      P->exported = exp;
    }
    X.leap_nsegs = 0;
    X.mark("epilogue launched");
  }
  if (P->mode == MODE_HASH && !P->part_hash && kp.pack_slot >= 0 &&
      launch_hash_unpack(X.table, kp.hash_keys, P->num_keys, kp.pack_slot, kp.pack_shift, stream))
    return fail(PGPU_ERR_DEVICE, "hash unpack launch failed: %s", hipGetErrorString(hipGetLastError()));
  if (X.leap_nsegs > 0 &&  // deferred but no fold ran (cannot happen for a plan with scan tiles; kept exact)
      launch_leap2_compose(X.leap_segs, P->seg_stride, X.leap_nsegs, kp.leap_maps, kp.stats, stream))
    return fail(PGPU_ERR_DEVICE, "filter statistics launch failed: %s", hipGetErrorString(hipGetLastError()));
  PGPU_TIMING_RECORD(P, sc->ev[3], stream);
  P->last_stream = stream;
  P->executed = true;
  if (trace_on()) {
    const double end = now_us();
    fprintf(stderr, "[pgpu] execute: %.1f us host\n", end - X.t_start);
    static const bool all_marks = diag("marks");  // PGPU_TRACE=1,marks: every execution's marks
    if (end - X.t_start > 1000.0 || all_marks) {
      double prev = X.t_start;
      for (const auto& m : X.marks) {
        fprintf(stderr, "[pgpu]   %s +%.1f us\n", m.first, m.second - prev);
        prev = m.second;
      }
      fprintf(stderr, "[pgpu]   (end) +%.1f us\n", end - prev);
    }
  }
  return 0;
}

int plan_execute_impl(pgpu_plan_s* P, hipStream_t stream, void* d_table) {
  const int nl = (int)P->chunks.size();
  ExecCtx X;
  TRY(exec_prologue(P, stream, d_table, std::max(nl, 1), X));
  for (int c = 0; c < nl; ++c) {
    TRY(exec_upload_chunk(P, stream, X, P->chunks[c]));
    TRY(exec_launch_chunk(P, stream, X, P->chunks[c], c));
  }
  return exec_epilogue(P, stream, X);
}

// Group-by dictIds of composite key k: (k / stride[j]) % card[j] (DictionaryBasedGroupKeyGenerator.java:276-323).
void decode_keys(const pgpu_plan_s* P, pgpu_result_s* R, int64_t row, uint64_t key) {
  for (int j = 0; j < R->num_keys; ++j)
    R->gid(j)[row] = (int32_t)((key / (uint64_t)P->key_stride[j]) % (uint64_t)P->key_card[j] + P->key_off[j]);
}

// key_begin / key_count: a shard [slots][key_count] of the dense table holding keys [key_begin, key_begin +
// key_count) (after a reduce-scatter across GPUs); the whole table is (0, num_keys).
int plan_finalize_impl(pgpu_plan_s* P, hipStream_t stream, const void* d_table, int64_t key_begin, int64_t key_count,
                       pgpu_result_s* R) {
  Scratch* sc = P->scratch;
  const double t_start = trace_on() ? now_us() : 0;
  if (!P->executed) return fail(PGPU_ERR_INVALID_ARGUMENT, "plan not executed");
  const uint64_t* table = reinterpret_cast<const uint64_t*>(d_table ? d_table : P->d_table_used);
  const int nslots = (int)P->slot_kind.size();
  const int nk = (int)P->key_cols.size();
  const int64_t G = key_count;
  int64_t n = 0;
  uint64_t matched = 0, star_scanned = 0;
  const int64_t words = (int64_t)nslots * G;
  // the epilogue wrote this execution's whole table + statistics to host memory, and nothing has changed the table
  // since (a combine clears P->exported)
  const bool from_export = P->exported && table == P->d_table_used && key_begin == 0 && G == P->num_keys;
  P->star_metric_bytes = -1;  // read back by the small-table path only
  double t_sync1 = 0;
  R->pool = P->table->result_pool;
  {
    // The buffers filled before the wait below: growing one frees the old one, and hipFree waits for the whole
    // device -- it would hold the wait (and a pgpu_plan_cancel or the query's deadline) until the scan is done.  When
    // one must grow, the plan's work is waited for first (cancel- and deadline-aware), then the buffers grow.
    bool grow = sc->counter.cap < 64 + (size_t)kMaxSlots * 16 || sc->readback.cap < 64 + (size_t)nslots * 16;
    if (!P->hash && words * 8 <= kHostCompactBytes && !from_export) grow |= sc->readback.cap < (size_t)words * 8 + 64;
    else if (!P->hash) grow |= sc->cslots.cap < compact_scratch_bytes(G, nslots);
    else if (!P->part_hash_live)
      grow |= sc->ckeys.cap < (size_t)std::max<int64_t>(1, std::min<int64_t>(G, P->merged_records >= 0
                                                                                 ? P->merged_records
                                                                                 : std::max<int64_t>(P->total_docs, 1))) *
                                 8 * (1 + nslots);
    if (grow) {
      TRY(wait_plan(P, stream));
      TRY(sc->counter.ensure(64 + (size_t)kMaxSlots * 16));
    }
  }
  if (!P->hash && words * 8 <= kHostCompactBytes) {
    // small dense table: the epilogue's copy in pinned host memory (from_export), else one or two copies (table +
    // stats) and one sync; compacted on the host in key order
    uint64_t* st;
    if (from_export) {
      st = reinterpret_cast<uint64_t*>(sc->exported.p);
    } else {
      TRY(sc->readback.ensure((size_t)words * 8 + 64));
      st = reinterpret_cast<uint64_t*>(sc->readback.p);
      if (reinterpret_cast<const uint8_t*>(P->d_stats) == reinterpret_cast<const uint8_t*>(table) + words * 8) {
        HIP_TRY(hipMemcpyAsync(st, table, (size_t)words * 8 + 64, hipMemcpyDeviceToHost, stream));  // table + stats
      } else {
        HIP_TRY(hipMemcpyAsync(st, table, (size_t)words * 8, hipMemcpyDeviceToHost, stream));
        HIP_TRY(hipMemcpyAsync(st + words, P->d_stats, 64, hipMemcpyDeviceToHost, stream));
      }
    }
    TRY(wait_plan(P, stream));
    t_sync1 = trace_on() ? now_us() : 0;
    if (st[words + 5]) return timeout_fail(P);
    matched = st[words];
    star_scanned = st[words + 1] + st[words + 2];
    P->star_docs_read = (int64_t)st[words + 3];
    P->star_metric_bytes = (int64_t)st[words + 7] * 64;
    for (int64_t k = 0; k < G; ++k) n += st[k] != 0;
    TRY(R->alloc(nk, nslots, n));
    int64_t j = 0;
    for (int64_t k = 0; k < G; ++k) {
      if (!st[k]) continue;
      decode_keys(P, R, j, (uint64_t)(key_begin + k));
      for (int s = 0; s < nslots; ++s) R->slot(s)[j] = st[(int64_t)s * G + k];
      ++j;
    }
  } else if (!P->hash) {
    // large dense table: ordered compaction on the device (count / scan, then a scatter in key order), copied back
    // into the pinned result buffer.  Two forms: the columnar dictIds + 8-byte words, or -- when it moves fewer
    // bytes, as for C5's 10M groups of 10M keys -- a presence bitmap over the keys plus each slot's words at the
    // narrowest width their range allows (decoded on the host on first access).
    const int64_t nch = compact_ordered_chunks(G);
    TRY(sc->counter.ensure(64 + (size_t)nslots * 16));
    TRY(sc->cslots.ensure(compact_scratch_bytes(G, nslots)));
    long long* d_minmax = reinterpret_cast<long long*>(sc->counter.as<uint8_t>() + 64);
    // K8d already counted this execution's table by chunk (unchanged since: no combine, the whole key range)
    const bool counted = P->k8d_counts && table == P->d_table_used && key_begin == 0 && G == P->num_keys;
    if (launch_compact_dense_count(table, nslots, G, sc->cslots.as<uint32_t>(), sc->counter.as<unsigned long long>(),
                                   d_minmax, stream, counted))
      return fail(PGPU_ERR_DEVICE, "compact count launch failed: %s", hipGetErrorString(hipGetLastError()));
    TRY(sc->readback.ensure(64 + (size_t)nslots * 16));
    uint64_t* st = reinterpret_cast<uint64_t*>(sc->readback.p);
    HIP_TRY(hipMemcpyAsync(st, sc->counter.p, 8, hipMemcpyDeviceToHost, stream));
    HIP_TRY(hipMemcpyAsync(st + 1, P->d_stats, 48, hipMemcpyDeviceToHost, stream));
    HIP_TRY(hipMemcpyAsync(st + 8, d_minmax, (size_t)nslots * 16, hipMemcpyDeviceToHost, stream));
    TRY(wait_plan(P, stream));
    t_sync1 = trace_on() ? now_us() : 0;
    if (st[6]) return timeout_fail(P);
    n = (int64_t)std::min<uint64_t>(st[0], (uint64_t)G);
    matched = st[1];
    star_scanned = st[2] + st[3];
    P->star_docs_read = (int64_t)st[4];
    std::vector<int32_t> width(nslots, 8);
    int64_t narrow_bytes = 0;
    for (int s = 0; s < nslots; ++s) {
      const long long lo = (long long)st[8 + s], hi = (long long)st[8 + nslots + s];
      width[s] = n > 0 ? compact_slot_width(lo, hi, P->slot_kind[s]) : 8;
      narrow_bytes += n * width[s];
    }
    const int64_t bitmap_words = (G + 63) / 64;
    const bool compact = P->cfg.compact_results && n > 0 && bitmap_words * 8 + narrow_bytes < n * (4 * nk + 8 * nslots);
    if (compact) {
      const int64_t cap = n;
      TRY(sc->ckeys.ensure((size_t)bitmap_words * 8 + (size_t)nslots * cap * 8));
      uint8_t* dev = sc->ckeys.as<uint8_t>();
      if (launch_compact_dense_scatter(table, nslots, G, P->slot_kind.data(), sc->cslots.as<uint32_t>(), d_minmax,
                                       reinterpret_cast<uint64_t*>(dev), dev + bitmap_words * 8, cap, stream))
        return fail(PGPU_ERR_DEVICE, "compact scatter launch failed: %s", hipGetErrorString(hipGetLastError()));
      R->num_keys = nk;
      R->num_slots = nslots;
      R->n = n;
      R->ckey_base = key_begin;
      R->cbits = G;
      R->cstride = P->key_stride;
      R->ccard = P->key_card;
      R->coff = P->key_off;
      R->cwidth = width;
      R->cslot_off.assign(nslots, 0);
      size_t off = (size_t)bitmap_words * 8;
      for (int s = 0; s < nslots; ++s) {
        R->cslot_off[s] = off;
        off += ((size_t)n * width[s] + 7) & ~size_t(7);
      }
      if (R->pool) R->cbuf = R->pool->take();
      TRY(R->cbuf.ensure(off));
      uint8_t* h = reinterpret_cast<uint8_t*>(R->cbuf.p);
      HIP_TRY(hipMemcpyAsync(h, dev, (size_t)bitmap_words * 8, hipMemcpyDeviceToHost, stream));
      for (int s = 0; s < nslots; ++s)
        HIP_TRY(hipMemcpyAsync(h + R->cslot_off[s], dev + bitmap_words * 8 + (size_t)s * cap * 8, (size_t)n * width[s],
                               hipMemcpyDeviceToHost, stream));
      HIP_TRY(hipStreamSynchronize(stream));
      R->compact.store(true, std::memory_order_release);
    } else {
      const int64_t cap = std::max<int64_t>(2, (n + 1) & ~int64_t(1));
      TRY(sc->ckeys.ensure((size_t)cap * (4 * nk + 8 * nslots) + 8));
      if (launch_compact_ordered_scatter(table, nslots, G, key_begin, P->key_stride.data(), P->key_card.data(),
                                         P->key_off.data(), nk, sc->cslots.as<uint32_t>(), sc->ckeys.p, cap, stream))
        return fail(PGPU_ERR_DEVICE, "compact launch failed: %s", hipGetErrorString(hipGetLastError()));
      TRY(R->alloc(nk, nslots, n));
      if (n > 0) {
        const uint8_t* dev = sc->ckeys.as<uint8_t>();
        for (int j = 0; j < nk; ++j)
          HIP_TRY(hipMemcpyAsync(R->gid_raw(j), dev + (size_t)j * cap * 4, (size_t)n * 4, hipMemcpyDeviceToHost, stream));
        for (int s = 0; s < nslots; ++s)
          HIP_TRY(hipMemcpyAsync(R->slot_raw(s), dev + (size_t)nk * cap * 4 + (size_t)s * cap * 8, (size_t)n * 8,
                                 hipMemcpyDeviceToHost, stream));
      }
      HIP_TRY(hipStreamSynchronize(stream));
    }
  } else {
    // hash table: unordered compaction, then key order on the host
    const int64_t rec = 1 + nslots;  // entry-major compact record: key, then the slot words
    int64_t cap;
    const bool k8h = P->part_hash_live;
    if (k8h) {  // K8h wrote the compacted records and their count at execute
      cap = part_hash_out_cap(P);
    } else {
      cap = std::max<int64_t>(1, std::min<int64_t>(G, P->merged_records >= 0 ? P->merged_records
                                                                            : std::max<int64_t>(P->total_docs, 1)));
      TRY(sc->counter.ensure(64));
      TRY(sc->ckeys.ensure((size_t)cap * 8 * rec));
      HIP_TRY(hipMemsetAsync(sc->counter.p, 0, 8, stream));
      if (launch_compact(table, sc->hash_keys.as<unsigned long long>(), nslots, G, sc->counter.as<unsigned long long>(),
                         sc->ckeys.as<uint64_t>(), cap, stream))
        return fail(PGPU_ERR_DEVICE, "compact launch failed");
    }
    // each slot's range over the records, read back with their count (the compact form's widths, below)
    const bool want_compact = P->stage_end.empty() && P->cfg.compact_results;
    TRY(sc->counter.ensure(64 + (size_t)kMaxSlots * 16));  // (no regrowth: the first allocation is 4 KB)
    unsigned long long* d_mm = reinterpret_cast<unsigned long long*>(sc->counter.as<uint8_t>() + 64);
    if (want_compact &&
        (k8h ? launch_hash_minmax_parts(sc->part_mm.as<unsigned long long>(), P->num_parts, nslots, d_mm, stream)
             : launch_hash_minmax(sc->ckeys.as<uint64_t>(), sc->counter.as<unsigned long long>(), cap, nslots, d_mm,
                                  stream)))
      return fail(PGPU_ERR_DEVICE, "slot range launch failed: %s", hipGetErrorString(hipGetLastError()));
    TRY(sc->readback.ensure(64 + (size_t)nslots * 16));
    uint64_t* st = reinterpret_cast<uint64_t*>(sc->readback.p);
    HIP_TRY(hipMemcpyAsync(st, sc->counter.p, 8, hipMemcpyDeviceToHost, stream));
    HIP_TRY(hipMemcpyAsync(st + 1, P->d_stats, 48, hipMemcpyDeviceToHost, stream));
    if (want_compact) HIP_TRY(hipMemcpyAsync(st + 8, d_mm, (size_t)nslots * 16, hipMemcpyDeviceToHost, stream));
    TRY(wait_plan(P, stream));
    t_sync1 = trace_on() ? now_us() : 0;
    if (st[6]) return timeout_fail(P);
    if (st[5])  // stats[4]: a probe found no free slot (hash_slot) -- the table was sized below the plan's groups
      return fail(PGPU_ERR_DEVICE, "group hash table of %lld slots overflowed (plan bound %lld groups)",
                  (long long)G, (long long)P->group_bound);
    if (k8h && st[0] > (uint64_t)cap) return part_hash_overflow(P, st[0]);
    n = (int64_t)std::min<uint64_t>(st[0], (uint64_t)cap);
    matched = st[1];
    star_scanned = st[2] + st[3];
    P->star_docs_read = (int64_t)st[4];
    if (P->groups_seen && P->merged_records < 0) P->groups_seen->store(n, std::memory_order_relaxed);
    if (n >= 4096 && P->stage_end.empty()) {
      // Decoded on the device in one streaming pass over the records, in their (hash / partition) order -- the
      // LONG_MAP holder's iteration order is fastutil's hash order (DictionaryBasedGroupKeyGenerator.java:693, :719)
      // and no consumer depends on group order -- held in compact form when that moves fewer bytes (C5-sized
      // results: 10M groups): composite keys at 4 or 8 bytes instead of the decoded dictIds, and each slot at the
      // narrowest width of its range (as the dense compact form); the host decodes it on first access
      // (result_expand).
      int key_bits = 1;
      {
        const long double space = (long double)P->key_stride[nk - 1] * (long double)P->key_card[nk - 1];
        while (key_bits < 64 && (long double)(INT64_C(1) << key_bits) < space) ++key_bits;
      }
      const int32_t key_width = key_bits <= 32 ? 4 : 8;
      std::vector<int32_t> width(nslots, 8);
      std::vector<int64_t> woff(nslots, 0);
      size_t cbytes = ((size_t)n * key_width + 7) & ~size_t(7);
      for (int s2 = 0; s2 < nslots; ++s2) {
        const long long lo = (long long)(st[8 + s2] ^ (1ull << 63)), hi = (long long)(st[8 + nslots + s2] ^ (1ull << 63));
        width[s2] = compact_slot_width(lo, hi, P->slot_kind[s2]);
        woff[s2] = (int64_t)cbytes;
        cbytes += ((size_t)n * width[s2] + 7) & ~size_t(7);
      }
      if (want_compact && cbytes < (size_t)n * (4 * nk + 8 * nslots)) {
        TRY(sc->hsort.ensure(cbytes + 256));
        uint8_t* out = sc->hsort.as<uint8_t>();
        if (launch_hash_compact(sc->ckeys.as<uint64_t>(), n, nslots, key_width, width.data(), woff.data(), out, stream))
          return fail(PGPU_ERR_DEVICE, "hash compact launch failed: %s", hipGetErrorString(hipGetLastError()));
        R->num_keys = nk;
        R->num_slots = nslots;
        R->n = n;
        R->ckey_width = key_width;
        R->cstride = P->key_stride;
        R->ccard = P->key_card;
        R->coff = P->key_off;
        R->cwidth = width;
        R->cslot_off.assign(woff.begin(), woff.end());
        if (R->pool) R->cbuf = R->pool->take();
        TRY(R->cbuf.ensure(cbytes));
        HIP_TRY(hipMemcpyAsync(R->cbuf.p, out, cbytes, hipMemcpyDeviceToHost, stream));
        HIP_TRY(hipStreamSynchronize(stream));
        R->compact.store(true, std::memory_order_release);
        n = -1;  // held compact
      }
    }
    if (n >= 4096 && P->stage_end.empty()) {
      // decoded into the columnar result on the device: one copy back
      const size_t slot_off = pgpu_result_s::slot_offset(nk, n);
      const size_t out_bytes = slot_off + (size_t)nslots * n * 8;
      TRY(sc->hsort.ensure(out_bytes + 256));
      uint8_t* out = sc->hsort.as<uint8_t>();
      if (launch_hash_decode(sc->ckeys.as<uint64_t>(), n, nslots, nk, P->key_stride.data(), P->key_card.data(),
                             P->key_off.data(), out, slot_off, stream))
        return fail(PGPU_ERR_DEVICE, "hash decode launch failed: %s", hipGetErrorString(hipGetLastError()));
      TRY(R->alloc(nk, nslots, n));
      HIP_TRY(hipMemcpyAsync(R->buf.p, out, out_bytes, hipMemcpyDeviceToHost, stream));
      HIP_TRY(hipStreamSynchronize(stream));
      n = -1;  // decoded
    } else if (n > 0) {
      TRY(sc->readback.ensure((size_t)n * rec * 8));
      st = reinterpret_cast<uint64_t*>(sc->readback.p);
      HIP_TRY(hipMemcpyAsync(st, sc->ckeys.p, (size_t)n * rec * 8, hipMemcpyDeviceToHost, stream));
      HIP_TRY(hipStreamSynchronize(stream));
    }
    if (n < 0) {
      n = R->n;
    } else {
    std::vector<uint64_t> stages;  // ARRAY_MAP: the stage tables (slot -> that group's key), back to back
    std::vector<int64_t> stage_off;
    if (!P->stage_end.empty() && n > 0) {
      int64_t total = 0;
      for (int64_t c : P->stage_cap) { stage_off.push_back(total); total += c; }
      stages.resize((size_t)total);
      HIP_TRY(hipMemcpyAsync(stages.data(), sc->stage_keys.p, (size_t)total * 8, hipMemcpyDeviceToHost, stream));
      HIP_TRY(hipStreamSynchronize(stream));
    }
    std::vector<int64_t> order(n);
    for (int64_t i = 0; i < n; ++i) order[i] = i;
    std::sort(order.begin(), order.end(), [&](int64_t a, int64_t b) { return st[a * rec] < st[b * rec]; });
    TRY(R->alloc(nk, nslots, n));
    for (int64_t r = 0; r < n; ++r) {
      const uint64_t* e = st + order[r] * rec;
      if (!P->stage_end.empty()) {  // last group first: its key's slot part names the previous group's key
        uint64_t cur = e[0];
        for (int g = (int)P->stage_space.size() - 1; g >= 0; --g) {
          const uint64_t local = cur % (uint64_t)P->stage_space[g], slot = cur / (uint64_t)P->stage_space[g];
          const int j0 = g == 0 ? 0 : P->stage_end[g - 1], j1 = g < (int)P->stage_end.size() ? P->stage_end[g] : nk;
          for (int j = j0; j < j1; ++j)
            R->gid(j)[r] = (int32_t)((local / (uint64_t)P->key_stride[j]) % (uint64_t)P->key_card[j]);
          if (g > 0) {
            if (slot >= (uint64_t)P->stage_cap[g - 1]) return fail(PGPU_ERR_DEVICE, "ARRAY_MAP stage slot out of range");
            cur = stages[(size_t)(stage_off[g - 1] + (int64_t)slot)];
          }
        }
      } else {
        decode_keys(P, R, r, e[0]);
      }
      for (int s = 0; s < nslots; ++s) R->slot(s)[r] = e[1 + s];
    }
    }
  }
  const double t_sync2 = trace_on() ? now_us() : 0;
  const int na = (int)P->agg_fn.size();
  R->num_aggs = na;
  R->agg_slot = P->agg_slot;
  R->slot_kind = P->slot_kind;
  R->key_cols = P->key_cols;
  R->key_dicts.assign(P->key_dicts.begin(), P->key_dicts.end());
  R->key_types.clear();
  for (int c : P->key_cols) R->key_types.push_back(P->table->types[c]);
  R->agg_fn = P->agg_fn;
  R->agg_col = P->agg_col;
  R->agg_conv.assign(na, RCONV_I64);
  for (int a = 0; a < na; ++a) {
    const int fn = P->agg_fn[a];
    if (fn == PGPU_AGG_COUNT) continue;  // CountAggregationFunction: exact count (held as double by Pinot)
    if (fn == PGPU_AGG_SUM || fn == PGPU_AGG_AVG)
      R->agg_conv[a] = P->slot_kind[P->agg_slot[a]] == SLOT_SUM_I64 ? RCONV_I64 : RCONV_F64;
    else
      R->agg_conv[a] = is_int_type(P->table->types[P->agg_col[a]]) ? RCONV_I64 : RCONV_KEY_F64;
  }
  int64_t generic_entries = 0;
  if (!P->generic.empty()) {  // the leaves' bitmaps were copied into maskstage by the (synchronised) stream
    const uint32_t* words = reinterpret_cast<const uint32_t*>(P->scratch->maskstage.p);
    std::vector<int64_t> part(P->generic.size(), 0);
    auto replay = [&](int i) {
      const auto& g = P->generic[i];
      const int64_t ngroups = ((int64_t)g.num_docs + 31) / 32;
      std::vector<const uint32_t*> masks(P->num_leaves);
      for (int k = 0; k < P->num_leaves; ++k) masks[P->leaf_perm[k]] = words + g.out_word + (int64_t)k * ngroups;
      part[i] = simulate_entries_scanned(g.tree, masks, g.num_docs);
    };
    if (P->generic.size() > 4) host_pool().run((int)P->generic.size(), replay);
    else for (size_t i = 0; i < P->generic.size(); ++i) replay((int)i);
    for (int64_t v : part) generic_entries += v;
  }
  // GroupByCombineOperator.mergeResults (:215-219): the merged map holds >= numGroupsLimit groups (PQL mode only)
  R->groups_limit_reached = P->pql_cap && nk > 0 && P->num_groups_limit > 0 && n >= P->num_groups_limit;
  R->stats[0] = (int64_t)matched;
  R->stats[1] = P->scanned_entries_model + (int64_t)star_scanned + generic_entries;
  R->stats[2] = ((int64_t)matched - P->post_exempt_docs) * P->num_projected;
  R->stats[3] = P->total_docs;
  R->stats[4] = (int64_t)P->segs.size();
  R->stats[5] = P->segments_matched_filter;
  if (trace_on())
    fprintf(stderr, "[pgpu] finalize: launch+sync1 %.1f us, copy+sync2 %.1f us, decode %.1f us (n=%lld)\n",
            t_sync1 - t_start, t_sync2 - t_sync1, now_us() - t_sync2, (long long)n);
  return 0;
}

}  // namespace pgpu

// Columnar form of a compact result: rows are the bitmap's set bits in key order; each block of 4096 bitmap words is
// decoded by one task of the host pool (a prefix of its popcounts gives its first row).
int pgpu::result_expand(pgpu_result_s* R) {
  std::lock_guard<std::mutex> g(R->expand_mu);
  if (!R->compact.load(std::memory_order_acquire)) return 0;
  const int nk = R->num_keys, ns = R->num_slots;
  const int64_t n = R->n;
  TRY(R->alloc(nk, ns, n));
  if (R->ckey_width) {  // composite keys (hash-mode results): decode each row's key
    const uint8_t* kb = reinterpret_cast<const uint8_t*>(R->cbuf.p);
    constexpr int64_t kRowsPerTask = 1 << 20;
    const int64_t ktasks = (n + kRowsPerTask - 1) / kRowsPerTask;
    auto keys = [&](int t) {
      const int64_t r0 = t * kRowsPerTask, r1 = std::min(n, r0 + kRowsPerTask);
      for (int64_t r = r0; r < r1; ++r) {
        const uint64_t key = R->ckey_width == 4 ? (uint64_t)reinterpret_cast<const uint32_t*>(kb)[r]
                                                : reinterpret_cast<const uint64_t*>(kb)[r];
        for (int j = 0; j < nk; ++j)
          R->gid_raw(j)[r] = (int32_t)((key / (uint64_t)R->cstride[j]) % (uint64_t)R->ccard[j] + R->coff[j]);
      }
    };
    if (ktasks > 1) host_pool().run((int)ktasks, keys);
    else if (ktasks == 1) keys(0);
  }
  const uint64_t* bm = reinterpret_cast<const uint64_t*>(R->cbuf.p);
  const int64_t words = R->ckey_width ? 0 : (R->cbits + 63) / 64;
  constexpr int64_t kBlockWords = 4096;
  const int64_t nb = (words + kBlockWords - 1) / kBlockWords;
  std::vector<int64_t> first(nb + 1, 0);
  auto count = [&](int b) {
    int64_t c = 0;
    for (int64_t w = b * kBlockWords; w < std::min(words, (b + 1) * kBlockWords); ++w) c += __builtin_popcountll(bm[w]);
    first[b + 1] = c;
  };
  auto decode = [&](int b) {
    int64_t row = first[b];
    std::vector<int32_t*> gid(nk);
    for (int j = 0; j < nk; ++j) gid[j] = R->gid_raw(j);
    for (int64_t w = b * kBlockWords; w < std::min(words, (b + 1) * kBlockWords); ++w) {
      for (uint64_t bits = bm[w]; bits; bits &= bits - 1, ++row) {
        if (row >= n) return;
        const uint64_t key = (uint64_t)(R->ckey_base + w * 64 + __builtin_ctzll(bits));
        for (int j = 0; j < nk; ++j)
          gid[j][row] = (int32_t)((key / (uint64_t)R->cstride[j]) % (uint64_t)R->ccard[j] + R->coff[j]);
      }
    }
  };
  if (nb > 1) host_pool().run((int)nb, count);
  else if (nb == 1) count(0);
  for (int64_t b = 0; b < nb; ++b) first[b + 1] += first[b];
  if (nb > 1) host_pool().run((int)nb, decode);
  else if (nb == 1) decode(0);
  // the words, sign-extended from their compact widths
  const uint8_t* base = reinterpret_cast<const uint8_t*>(R->cbuf.p);
  constexpr int64_t kRows = 1 << 20;
  const int64_t tasks = (n + kRows - 1) / kRows;
  auto widen = [&](int t) {
    const int64_t r0 = t * kRows, r1 = std::min(n, r0 + kRows);
    for (int s = 0; s < ns; ++s) {
      const uint8_t* src = base + R->cslot_off[s];
      uint64_t* dst = R->slot_raw(s);
      switch (R->cwidth[s]) {
        case 1: for (int64_t r = r0; r < r1; ++r) dst[r] = (uint64_t)(int64_t)reinterpret_cast<const int8_t*>(src)[r]; break;
        case 2: for (int64_t r = r0; r < r1; ++r) dst[r] = (uint64_t)(int64_t)reinterpret_cast<const int16_t*>(src)[r]; break;
        case 3:  // 24-bit little-endian, sign-extended
          for (int64_t r = r0; r < r1; ++r) {
            const uint32_t u = (uint32_t)src[3 * r] | (uint32_t)src[3 * r + 1] << 8 | (uint32_t)src[3 * r + 2] << 16;
            dst[r] = (uint64_t)(int64_t)((int32_t)(u << 8) >> 8);
          }
          break;
        case 4: for (int64_t r = r0; r < r1; ++r) dst[r] = (uint64_t)(int64_t)reinterpret_cast<const int32_t*>(src)[r]; break;
        default: memcpy(dst + r0, reinterpret_cast<const uint64_t*>(src) + r0, (size_t)(r1 - r0) * 8); break;
      }
    }
  };
  if (tasks > 1) host_pool().run((int)tasks, widen);
  else if (tasks == 1) widen(0);
  R->compact.store(false, std::memory_order_release);
  return 0;
}

