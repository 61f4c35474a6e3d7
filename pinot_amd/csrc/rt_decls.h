// rt_decls.h -- prototypes of the functions and variables the runtime's sources share (see rt.h).
#pragma once
#include "rt.h"

namespace pgpu {

// rt_core.cpp
void crash_trace_handler(int sig, siginfo_t* si, void* uc);
bool diag(const char* word);
void install_crash_trace();
extern thread_local std::string g_err;
bool trace_on();
double now_us();
int fail(int code, const char* fmt, ...);

// rt_dict.cpp
int parse_dictionary(int type, const pgpu_column_buffers& cb, Dict* d);
bool dbl_less(double a, double b);
bool merge_dict(std::shared_ptr<const Dict>& g, const Dict& src);
int64_t global_index_of(const Dict& g, const Dict& local, size_t i);
int ensure_lut(pgpu_table_s* t, Segment& s, int col, hipStream_t stream);
int ensure_values(pgpu_table_s* t, Segment& s, int col, hipStream_t stream);
int ensure_global_values(pgpu_table_s* t, int col, hipStream_t stream);
int ensure_value_map(pgpu_table_s* t, Segment& s, int col);
int ensure_docid(pgpu_table_s* t, int64_t n, hipStream_t stream);
void account_unpin(pgpu_table_s* t, const Segment* s);
int64_t padded_fwd_words(int64_t num_docs, int bits);
int64_t lz4_decode_block(const uint8_t* src, int64_t n, uint8_t* dst, int64_t cap);
int decode_raw_forward_index(int type, const uint8_t* b, int64_t n, int32_t num_docs, int c, RawValues* out);
int parse_raw_column(int type, const pgpu_column_buffers& cb, int32_t num_docs, int c, Column* col, RawValues* out);
int64_t register_segment(pgpu_table_s* t, std::unique_ptr<Segment> seg_in);

// rt_plan.cpp
int64_t hash_capacity(int64_t groups);
Scratch* acquire_scratch(pgpu_table_s* t);
void release_scratch(pgpu_table_s* t, Scratch* s);
bool parse_literal(int type, const char* lit, bool allow_star, Literal* out);
int insertion_index(const Column& c, const Literal& v);
int parse_predicate(int type, const pgpu_predicate& p, ParsedPred* out);
void to_inverted_leaf(const Column& c, const pgpu_predicate& p, const Segment& s, LeafHost* L);
int translate_predicate(const Column& c, const pgpu_predicate& p, const ParsedPred& pp, LeafHost* L,
                        std::vector<int>& ids);
int translate_predicate_dict(const Column& c, const pgpu_predicate& p, const ParsedPred& pp, LeafHost* L,
                             std::vector<int>& ids);
void translate_raw_predicate(int type, const pgpu_predicate& p, const ParsedPred& pp, LeafHost* L);
double estimate_selectivity(const std::vector<int32_t>& ops, const std::vector<double>& leaf);
Tri fold_program(const std::vector<int32_t>& ops, const std::vector<Tri>& leaf);
bool star_composites(const std::vector<int32_t>& ops, const pgpu_query* q, std::vector<std::vector<int>>* out);
void leaf_bitset(const LeafHost& L, int32_t card, std::vector<uint32_t>& w);
int plan_star_segment(pgpu_plan_s* P, size_t seg_index, Segment* s, const pgpu_query* q,
                      const std::vector<std::vector<int>>& comps, const std::vector<LeafHost>& leaves, bool* used);
SegStats classify_segment_stats(const pgpu_plan_s* P, uint64_t sig);
bool int_sum_fits(const std::vector<Segment*>& segs, int col);
int32_t pack_slot_for(const pgpu_table_s* t, const pgpu_plan_s* P, const pgpu_query* q, int64_t max_count,
                      int shift);
int32_t lds_pack_slot(const pgpu_table_s* t, const pgpu_plan_s* P, const pgpu_query* q, int64_t G);
int32_t hash_pack_slot(const pgpu_table_s* t, const pgpu_plan_s* P, const pgpu_query* q, int* shift);
bool part_hash_eligible(const pgpu_plan_s* P, int64_t G);
void hash_part_bits(const pgpu_config& cfg, int64_t groups, int nslots, int* pbits, int* sbits);
int part_coarse_shift(int num_parts);
int part_coarse_runs(int num_parts);
void hash_part_resize(pgpu_plan_s* P, int64_t groups);
int64_t part_hash_out_cap(const pgpu_plan_s* P);
int part_hash_overflow(const pgpu_plan_s* P, uint64_t groups);
int plan_create_impl(pgpu_table_s* t, const int64_t* handles, int32_t nsegs, const pgpu_query* q, pgpu_plan_s* P,
                     const StreamExec* se = nullptr);

// rt_exec.cpp
double epoch_us();
int deadline_ticks(pgpu_table_s* t, int64_t end_ms, uint64_t* out);
int timeout_fail(const pgpu_plan_s* P);
int abandon_scratch(Scratch* sc, hipStream_t stream);
int cancel_fail();
bool cancelled(const pgpu_plan_s* P);
int wait_plan(pgpu_plan_s* P, hipStream_t stream);
int launch_raw_leaves(const pgpu_plan_s* P, Scratch* sc, hipStream_t stream);
void dense_lds_forms(const pgpu_plan_s* P, int32_t* pack_slot, uint32_t* narrow);
int exec_prologue(pgpu_plan_s* P, hipStream_t stream, void* d_table, int max_chunks, ExecCtx& X);
int exec_upload_chunk(pgpu_plan_s* P, hipStream_t stream, const ExecCtx& X, const LaunchChunk& C);
bool check_launch_on();
int check_launch_inputs(const pgpu_plan_s* P, hipStream_t stream, const ExecCtx& X, const LaunchChunk& C);
int scan_variant(const pgpu_plan_s* P);
extern unsigned long long* g_diag_times;
int diag_wg_times_begin(KParams& kp, int grid, hipStream_t stream);
int diag_wg_times_report(pgpu_table_s* t, const KParams& kp, int grid, hipStream_t stream);
void set_tile_claims(KParams& kp, unsigned long long* d_stats, int grid, int launch);
void set_slot_weights(KParams& kp, int grid, int num_cus, double step);
void inflight_begin(pgpu_plan_s* P);
void inflight_end(pgpu_plan_s* P);
int exec_launch_chunk(pgpu_plan_s* P, hipStream_t stream, ExecCtx& X, const LaunchChunk& C, int c);
int exec_epilogue(pgpu_plan_s* P, hipStream_t stream, ExecCtx& X);
int plan_execute_impl(pgpu_plan_s* P, hipStream_t stream, void* d_table);
void decode_keys(const pgpu_plan_s* P, pgpu_result_s* R, int64_t row, uint64_t key);
int plan_finalize_impl(pgpu_plan_s* P, hipStream_t stream, const void* d_table, int64_t key_begin, int64_t key_count,
                       pgpu_result_s* R);

// rt_groups.cpp
int split_for_groups_limit(pgpu_table_s* t, const int64_t* handles, int32_t nsegs, const pgpu_query* q,
                           pgpu_plan_s* P, bool* composite);
int composite_finalize(pgpu_plan_s* P, hipStream_t stream, pgpu_result_s* R);
bool plan_cache_enabled(const pgpu_table_s* t, const pgpu_query* q);
std::string plan_cache_key(pgpu_table_s* t, const int64_t* handles, int32_t nsegs, const pgpu_query* q);
bool plan_cache_get(pgpu_table_s* t, const std::string& key, pgpu_plan_s* P);
void plan_cache_clear(pgpu_table_s* t);
void plan_cache_put(pgpu_table_s* t, const std::string& key, pgpu_plan_s& P);

}  // namespace pgpu

