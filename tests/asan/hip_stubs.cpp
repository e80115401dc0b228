// Stand-in HIP runtime for the host-only sanitizer build of the C ABI (tests/test_asan_abi.py).
// The library's objects are compiled with --offload-host-only, so they carry no device code;
// linking them against these stubs instead of libamdhip64 keeps the run independent of any
// GPU or driver.  Every device operation fails with hipErrorNoDevice and is counted: the
// argument checks under test must reject their inputs before any launch or memory operation
// (hip_stub_device_ops() must read 0 at the end).  Test infrastructure only.
#include <hip/hip_runtime.h>

static int g_device_ops = 0;

extern "C" int hip_stub_device_ops(void) { return g_device_ops; }

extern "C" {
void** __hipRegisterFatBinary(const void*) {
    static void* handle = nullptr;
    return &handle;
}
void __hipUnregisterFatBinary(void**) {}
void __hipRegisterFunction(void**, const void*, char*, const char*, unsigned int, uint3*, uint3*, dim3*, dim3*,
                           int*) {}
void __hipRegisterVar(void**, void*, char*, char*, int, size_t, int, int) {}
hipError_t __hipPushCallConfiguration(dim3, dim3, size_t, hipStream_t) { return hipSuccess; }
hipError_t __hipPopCallConfiguration(dim3*, dim3*, size_t*, hipStream_t*) { return hipSuccess; }
}

hipError_t hipLaunchKernel(const void*, dim3, dim3, void**, size_t, hipStream_t) {
    ++g_device_ops;
    return hipErrorNoDevice;
}
hipError_t hipMemsetAsync(void*, int, size_t, hipStream_t) {
    ++g_device_ops;
    return hipErrorNoDevice;
}
hipError_t hipMemcpyAsync(void*, const void*, size_t, hipMemcpyKind, hipStream_t) {
    ++g_device_ops;
    return hipErrorNoDevice;
}
hipError_t hipMemcpy2DAsync(void*, size_t, const void*, size_t, size_t, size_t, hipMemcpyKind, hipStream_t) {
    ++g_device_ops;
    return hipErrorNoDevice;
}
hipError_t hipMemcpyFromSymbol(void*, const void*, size_t, size_t, hipMemcpyKind) {
    ++g_device_ops;
    return hipErrorNoDevice;
}
hipError_t hipGetDevice(int*) { return hipErrorNoDevice; }
hipError_t hipStreamIsCapturing(hipStream_t, hipStreamCaptureStatus* s) {
    if (s) *s = hipStreamCaptureStatusNone;
    return hipErrorNoDevice;
}
hipError_t hipDeviceGetAttribute(int*, hipDeviceAttribute_t, int) { return hipErrorNoDevice; }
hipError_t hipEventCreate(hipEvent_t*) { return hipErrorNoDevice; }
hipError_t hipEventDestroy(hipEvent_t) { return hipErrorNoDevice; }
hipError_t hipEventRecord(hipEvent_t, hipStream_t) { return hipErrorNoDevice; }
hipError_t hipEventElapsedTime(float*, hipEvent_t, hipEvent_t) { return hipErrorNoDevice; }
hipError_t hipGetLastError(void) { return hipSuccess; }
const char* hipGetErrorString(hipError_t) { return "no device (host-only sanitizer build)"; }
