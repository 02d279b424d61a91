// hg_launch.hpp -- kernel launches that report their own status.
#pragma once

#include <hip/hip_runtime.h>

#include <utility>

namespace hg {

// Launches `kernel` on `stream` and returns the status of THIS launch.
//
// hipLaunchKernel returns the launch's own status.  The `<<<>>>` form returns nothing, and
// a hipGetLastError() after it would also report -- and consume -- an error that an
// unrelated earlier HIP call left pending on the calling thread (a caller's failed
// hipMalloc would turn a valid solve into a failure).  Launching this way leaves such a
// pending error where it was, for its owner to read.
template <typename... KArgs, typename... Args>
inline int launch(void (*kernel)(KArgs...), dim3 grid, dim3 block, size_t lds, hipStream_t stream,
                  Args&&... args) {
    static_assert(sizeof...(KArgs) == sizeof...(Args), "kernel argument count");
    return [&](KArgs... a) {
        void* p[] = {(void*)&a...};
        return (int)hipLaunchKernel(reinterpret_cast<const void*>(kernel), grid, block, p, lds,
                                    stream);
    }(std::forward<Args>(args)...);
}

}  // namespace hg
