// kf_internal.h -- shared helpers of the kf2vec_gpu library (not part of the ABI).
#pragma once
#include <mutex>
#include <stdint.h>

#include "../../include/kf2vec_gpu.h"

// Records the thread-local error message and returns `code`.
int kf_fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));


// kf_read_files with a progress callback (kf_host.cpp): ready(lo, hi, ctx) gets
// consecutive ranges of dst, off[0]..off[n], once all their bytes are in place,
// in order and one at a time, each >= group bytes but the last; a nonzero
// return fails the call.
int kf_read_files_cb(const char* const* paths, int32_t n, const uint64_t* sizes, const uint64_t* off,
                     uint8_t* dst, uint64_t piece, int n_threads, uint64_t group,
                     int (*ready)(uint64_t lo, uint64_t hi, void* ctx), void* ctx);
