// include/compat/smallz4.h -- same file name as the reference's header, for code that does
// `#include "smallz4.h"`: put include/compat and include/ on the include path and link
// libsmallz4_amd.so, and smallz4::lz4(...) runs on the MI355X.
#pragma once
#include "../smallz4_amd.hpp"
