// host_common.h — host-side helpers shared by the runtime's translation units (not part of the ABI).
#pragma once

namespace pgpu {

// Records `fmt` as the calling thread's last error (pgpu_last_error) and returns `code`.
int host_fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));

// No C++ exception leaves an extern "C" entry point (a JNI or ctypes caller would abort): every ABI function body is
// a function-try-block ending in PGPU_ABI_CATCH, which maps std::bad_alloc to PGPU_ERR_OUT_OF_MEMORY and anything
// else to PGPU_ERR_INVALID_ARGUMENT, with the message as the thread's last error.  Call only inside a handler.
int abi_exception() noexcept;

}  // namespace pgpu

#define PGPU_ABI_CATCH \
  catch (...) {        \
    return pgpu::abi_exception(); \
  }

namespace pgpu {

}  // namespace pgpu
