// host_common.h — host-side helpers shared by the runtime's translation units (not part of the ABI).
#pragma once

namespace pgpu {

// Records `fmt` as the calling thread's last error (pgpu_last_error) and returns `code`.
int host_fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));

}  // namespace pgpu
