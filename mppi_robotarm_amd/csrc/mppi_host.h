// mppi_host.h — host-side helpers shared by the translation units of
// libmppi_rocm.so (one error channel behind mppi_last_error()).
#pragma once

#include <string>

namespace mppi_host {

// Records msg as this thread's last error (mppi_last_error) and returns code.
int fail(int code, const std::string& msg);

// The in-launch exchange's poll bound in s_memrealtime ticks (10 ns): MPPI_EXCHANGE_TIMEOUT_US when set
// (tests bound it to milliseconds), else 0 (the device's spin bound, ~1 s).
unsigned exchange_timeout_ticks();

}  // namespace mppi_host
