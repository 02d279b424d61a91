// sks_aca_sks.hpp -- drop-in for the reference's C++ solver interface
// (C++ Codes/modules/ACA_SKS.hpp:8-22, namespace sks), served by the MI355X kernels.
//
// The four single-problem functions keep the reference's exact signatures and
// output semantics (normalised H, H[8] == 1, bit-identical values).  The pointers
// may be host memory -- the reference's one-call-per-homography use in
// CPU_Runtime Test/main.cpp:87-114: the 16 values ride in the kernel launch
// and H comes back through per-thread mapped host memory on a per-thread stream, the
// thread spinning on a completion word the kernel writes after H (~9 us per call) -- or
// device memory (solved in place, on the legacy default stream).  The call is
// synchronous, as the reference's is, and thread-safe.
// Returns 0 on success (the reference always returns 0, ACA_SKS.cpp:101), or the
// hipError_t of a failed copy/launch.
//
// The *_batch overloads are the bulk entry points a caller should use: AoS
// (n,8)/(n,8)/(n,9), normalised.  Device-visible buffers (device, managed or pinned host
// memory) are solved asynchronously on `stream` (hipStream_t or NULL); if any buffer is
// pageable host memory the call goes through hg_solve_host_* (copied through the library's
// ring of pinned stages -- the caller's pages are never mapped for the GPU -- synchronous).
#pragma once
#include <cstdint>

#include "sks_homography.h"

namespace sks {

int runKernel_ACA(float* src, float* tar, float* result);          // ACA_SKS.hpp:17
int runKernel_ACA_double(double* src, double* tar, double* result); // ACA_SKS.hpp:18
int runKernel_SKS(float* src, float* tar, float* result);          // ACA_SKS.hpp:19
int runKernel_SKS_double(double* src, double* tar, double* result); // ACA_SKS.hpp:20

int runKernel_ACA_batch(const float* src, const float* tar, float* result, int64_t n,
                        void* stream = nullptr);
int runKernel_ACA_double_batch(const double* src, const double* tar, double* result,
                               int64_t n, void* stream = nullptr);
int runKernel_SKS_batch(const float* src, const float* tar, float* result, int64_t n,
                        void* stream = nullptr);
int runKernel_SKS_double_batch(const double* src, const double* tar, double* result,
                               int64_t n, void* stream = nullptr);

}  // namespace sks
