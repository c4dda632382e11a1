// dab_internal.h — shared declarations of the MI355X BA library (not part of the ABI).
#pragma once
#include <cstdint>
#include <string>

#include "../../include/dab.h"

namespace dab {

// Thread-local last error (dab_last_error). Returns `code` for `return set_error(...)`.
int set_error(int code, const std::string& msg);
void clear_error();

}  // namespace dab
