// rt_core.cpp -- errors, diagnostics and the table-config / dictionary views of the host runtime (rt.h).
#include "rt_decls.h"

// ================================================================================================ errors
namespace pgpu {

// PGPU_TRACE=crash (diagnostics): on SIGSEGV / SIGBUS / SIGABRT print the faulting address and the native frames
// (backtrace_symbols_fd: object, symbol or offset -- resolve offsets with addr2line -f -C -e <object>), then hand the
// signal to the previously installed handler (Python's faulthandler prints the Python stacks).
struct sigaction g_prev_segv, g_prev_bus, g_prev_abrt;
void crash_trace_handler(int sig, siginfo_t* si, void* uc) {
  char line[160];
  int len = snprintf(line, sizeof line, "[pgpu] fatal signal %d at address %p (thread %lu)\n", sig,
                     si ? si->si_addr : nullptr, (unsigned long)pthread_self());
  if (len > 0) { ssize_t w = write(2, line, (size_t)len); (void)w; }
  void* frames[64];
  const int n = backtrace(frames, 64);
  backtrace_symbols_fd(frames, n, 2);
  for (int i = 0; i < n; ++i) {  // offsets into their objects, for addr2line
    Dl_info info;
    if (dladdr(frames[i], &info) && info.dli_fname) {
      len = snprintf(line, sizeof line, "[pgpu]   #%d %s +0x%lx\n", i, info.dli_fname,
                     (unsigned long)((uintptr_t)frames[i] - (uintptr_t)info.dli_fbase));
      if (len > 0) { ssize_t w = write(2, line, (size_t)len); (void)w; }
    }
  }
  const struct sigaction* prev = sig == SIGSEGV ? &g_prev_segv : sig == SIGBUS ? &g_prev_bus : &g_prev_abrt;
  if (prev->sa_flags & SA_SIGINFO) {
    if (prev->sa_sigaction) { prev->sa_sigaction(sig, si, uc); return; }
  } else if (prev->sa_handler != SIG_DFL && prev->sa_handler != SIG_IGN && prev->sa_handler) {
    prev->sa_handler(sig);
    return;
  }
  signal(sig, SIG_DFL);
  raise(sig);
}
// Diagnostics: PGPU_TRACE, the one environment variable the library reads -- comma-separated words, none of which
// changes a result: "1" (per-phase host times of every plan, execution and finalize on stderr), "crash" (on
// SIGSEGV / SIGBUS / SIGABRT print the native frames), "check" (a scan launch's records and tile map are read back
// and checked before the launch), "serialize" (entry points run one at a time: isolates host races from device ones).
// Executor settings are pgpu_config's (pgpu_table_set_config), never the environment.
bool diag(const char* word) {
  static const std::string v = [] {
    const char* e = getenv("PGPU_TRACE");
    return "," + std::string(e ? e : "") + ",";
  }();
  return v.find("," + std::string(word) + ",") != std::string::npos;
}

struct CrashTraceInstaller {
  void install() {
    if (!diag("crash")) return;
    void* warm[2];
    backtrace(warm, 2);  // loads the unwinder now, not inside the handler
    struct sigaction sa;
    memset(&sa, 0, sizeof sa);
    sa.sa_sigaction = crash_trace_handler;
    sa.sa_flags = SA_SIGINFO | SA_ONSTACK;
    sigemptyset(&sa.sa_mask);
    sigaction(SIGSEGV, &sa, &g_prev_segv);
    sigaction(SIGBUS, &sa, &g_prev_bus);
    sigaction(SIGABRT, &sa, &g_prev_abrt);
    static const char msg[] = "[pgpu] crash trace installed\n";
    ssize_t w = write(2, msg, sizeof msg - 1);
    (void)w;
  }
};
void install_crash_trace() {
  static std::once_flag once;
  std::call_once(once, [] { CrashTraceInstaller().install(); });
}

thread_local std::string g_err;

// PGPU_TRACE=1: per-phase host timings on stderr (diagnostics only).
bool trace_on() {
  static const bool on = diag("1");
  return on;
}
double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int fail(int code, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

}  // namespace pgpu

int pgpu::host_fail(int code, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

int pgpu::abi_exception() noexcept {
  try {
    throw;
  } catch (const std::bad_alloc&) {
    g_err = "host allocation failed";
    return PGPU_ERR_OUT_OF_MEMORY;
  } catch (const std::exception& e) {
    return host_fail(PGPU_ERR_INVALID_ARGUMENT, "internal error: %s", e.what());
  } catch (...) {
    return host_fail(PGPU_ERR_INVALID_ARGUMENT, "internal error");
  }
}


int pgpu::table_dict_view(pgpu_table t, int col, DictView* out) {
  if (!t || col < 0 || col >= (int)t->names.size()) return host_fail(PGPU_ERR_INVALID_ARGUMENT, "bad column %d", col);
  std::shared_ptr<const Dict> d;
  {
    std::lock_guard<std::mutex> g(t->mu);
    d = t->global[col];
  }
  out->keep = d;
  out->type = d->type;
  out->iv = &d->iv;
  out->dv = &d->dv;
  out->sv = &d->sv;
  out->name = t->names[col];
  return 0;
}

int pgpu::result_key_dict_view(const pgpu_result_s* r, pgpu_table t, int key, DictView* out) {
  if (!r || key < 0 || key >= r->num_keys) return host_fail(PGPU_ERR_INVALID_ARGUMENT, "bad group-by key %d", key);
  if ((int)r->key_dicts.size() <= key || !r->key_dicts[key]) return table_dict_view(t, r->key_cols[key], out);
  auto d = std::static_pointer_cast<const Dict>(r->key_dicts[key]);
  out->keep = d;
  out->type = d->type;
  out->iv = &d->iv;
  out->dv = &d->dv;
  out->sv = &d->sv;
  out->name = t && r->key_cols[key] >= 0 && r->key_cols[key] < (int)t->names.size() ? t->names[r->key_cols[key]] : "";
  return 0;
}

pgpu_config table_config(const pgpu_table_s* t) {
  std::lock_guard<std::mutex> g(t->cfg_mu);
  return t->cfg;
}

