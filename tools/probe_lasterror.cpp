// probe_lasterror.cpp -- how HIP's per-thread last error behaves around the calls the C ABI
// makes (tools only; run on the GPU box by tools/gpu_round.sh lasterror):
//   1. does a failed hipSetDevice leave an error pending, and does a later successful call
//      (hipLaunchKernel, hipPointerGetAttributes on device memory) overwrite it?
//   2. which pointer queries fail on unregistered (pageable) host memory, and do they
//      overwrite a pending error?
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

__global__ void noop(int* p) {
    if (p && threadIdx.x == 0) *p = 1;
}

static const char* name(hipError_t e) { return hipGetErrorName(e); }

int main() {
    int* d = nullptr;
    if (hipMalloc(&d, 64) != hipSuccess) return 2;
    void* pageable = std::malloc(1 << 20);

    // 1. a pending error across a successful launch
    hipError_t e = hipSetDevice(9999);
    std::printf("setdevice(9999) -> %s; peek -> %s\n", name(e), name(hipPeekAtLastError()));
    void* args[] = {&d};
    e = hipLaunchKernel(reinterpret_cast<const void*>(noop), dim3(1), dim3(64), args, 0, nullptr);
    std::printf("hipLaunchKernel -> %s; peek after -> %s\n", name(e), name(hipPeekAtLastError()));
    noop<<<1, 64>>>(d);
    std::printf("<<<>>>; peek after -> %s\n", name(hipPeekAtLastError()));
    (void)hipGetLastError();

    // 2. pointer queries on pageable memory
    hipPointerAttribute_t a{};
    (void)hipSetDevice(9999);
    e = hipPointerGetAttributes(&a, d);
    std::printf("hipPointerGetAttributes(device) -> %s type %d; peek -> %s\n", name(e), (int)a.type,
                name(hipPeekAtLastError()));
    e = hipPointerGetAttributes(&a, pageable);
    std::printf("hipPointerGetAttributes(pageable) -> %s; peek -> %s\n", name(e),
                name(hipPeekAtLastError()));
    (void)hipGetLastError();
    (void)hipSetDevice(9999);
    unsigned int mt = 12345;
    e = hipPointerGetAttribute(&mt, HIP_POINTER_ATTRIBUTE_MEMORY_TYPE,
                               reinterpret_cast<hipDeviceptr_t>(pageable));
    std::printf("hipPointerGetAttribute(MEMORY_TYPE, pageable) -> %s value %u; peek -> %s\n",
                name(e), mt, name(hipPeekAtLastError()));
    (void)hipGetLastError();
    (void)hipSetDevice(9999);
    hipPointer_attribute at[1] = {HIP_POINTER_ATTRIBUTE_MEMORY_TYPE};
    mt = 12345;
    void* data[1] = {&mt};
    e = hipDrvPointerGetAttributes(1, at, data, reinterpret_cast<hipDeviceptr_t>(pageable));
    std::printf("hipDrvPointerGetAttributes(MEMORY_TYPE, pageable) -> %s value %u; peek -> %s\n",
                name(e), mt, name(hipPeekAtLastError()));
    mt = 12345;
    e = hipDrvPointerGetAttributes(1, at, data, reinterpret_cast<hipDeviceptr_t>(d));
    std::printf("hipDrvPointerGetAttributes(MEMORY_TYPE, device) -> %s value %u; peek -> %s\n",
                name(e), mt, name(hipPeekAtLastError()));
    (void)hipGetLastError();
    std::free(pageable);
    (void)hipFree(d);
    std::printf("probe done\n");
    return 0;
}
