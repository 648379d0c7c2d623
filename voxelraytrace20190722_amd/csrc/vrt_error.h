// vrt_error.h -- the thread-local error string behind vrt_last_error(),
// shared by every translation unit of libvrt.so (hidden symbol).
#pragma once

namespace vrt {
// Formats the message for vrt_last_error() and returns `code`.
int set_error(int code, const char *fmt, ...) __attribute__((format(printf, 2, 3)));
}  // namespace vrt
