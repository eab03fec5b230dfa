// orbx_error.h -- thread-local last-error string shared by the ABI translation units.
#pragma once

#include <string>

namespace orbx {
void set_last_error(const std::string& msg);
}
