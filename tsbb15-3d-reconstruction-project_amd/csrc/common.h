// Shared host-side helpers: status codes, thread-local error text.
#pragma once

#include <cstdarg>
#include <cstdio>
#include <string>

#include "rsamd.h"

namespace rs {

void set_error(const char *fmt, ...);

inline int fail(int code, const char *msg) {
  set_error("%s", msg);
  return code;
}

}  // namespace rs
