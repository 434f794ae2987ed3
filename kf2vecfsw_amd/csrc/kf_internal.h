// kf_internal.h -- shared helpers of the kf2vec_gpu library (not part of the ABI).
#pragma once
#include <mutex>
#include <stdint.h>

#include "../../include/kf2vec_gpu.h"

// Records the thread-local error message and returns `code`.
int kf_fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));

