// TEST INFRASTRUCTURE — a CPU stand-in for the slice of the HIP runtime API that kp_host.cpp (the C-ABI host layer of
// libkpsim) uses.  It is first on the include path only when tests/cpu_stub/Makefile compiles kp_host.cpp with g++
// (-fsanitize=thread) for the concurrency test; the product build (karpenter-provider-aws_amd/Makefile, hipcc) never
// sees it.  "Device memory" is host memory, streams are synchronous, the device count comes from KP_STUB_DEVICES.
#pragma once
#include <cstddef>
#include <cstdint>

typedef enum hipError_t { hipSuccess = 0, hipErrorInvalidValue = 1, hipErrorOutOfMemory = 2, hipErrorNoDevice = 100,
                          hipErrorInvalidDevice = 101 } hipError_t;
typedef enum hipMemcpyKind { hipMemcpyHostToHost = 0, hipMemcpyHostToDevice = 1, hipMemcpyDeviceToHost = 2,
                             hipMemcpyDeviceToDevice = 3, hipMemcpyDefault = 4 } hipMemcpyKind;
typedef struct ihipStream_t* hipStream_t;
typedef struct ihipEvent_t* hipEvent_t;
#define hipStreamNonBlocking 0x01

typedef struct hipDeviceProp_t {
    char name[256];
    char gcnArchName[256];
    size_t totalGlobalMem;
    int multiProcessorCount;
} hipDeviceProp_t;

struct int4 {
    int x, y, z, w;
};
inline int4 make_int4(int x, int y, int z, int w) { return int4{x, y, z, w}; }
struct int2 {
    int x, y;
};
inline int2 make_int2(int x, int y) { return int2{x, y}; }

hipError_t hipGetDeviceCount(int* n);
hipError_t hipSetDevice(int d);
hipError_t hipGetDeviceProperties(hipDeviceProp_t* p, int d);
const char* hipGetErrorString(hipError_t e);
hipError_t hipMalloc(void** p, size_t bytes);
hipError_t hipFree(void* p);
#define hipHostMallocDefault 0x0
hipError_t hipHostMalloc(void** p, size_t bytes, unsigned flags);
hipError_t hipHostFree(void* p);
hipError_t hipMemcpy(void* dst, const void* src, size_t bytes, hipMemcpyKind k);
hipError_t hipMemcpyAsync(void* dst, const void* src, size_t bytes, hipMemcpyKind k, hipStream_t s);
hipError_t hipMemsetAsync(void* dst, int v, size_t bytes, hipStream_t s);
hipError_t hipStreamCreateWithFlags(hipStream_t* s, unsigned flags);
hipError_t hipStreamDestroy(hipStream_t s);
hipError_t hipStreamSynchronize(hipStream_t s);
hipError_t hipEventCreate(hipEvent_t* e);
hipError_t hipEventDestroy(hipEvent_t e);
hipError_t hipEventRecord(hipEvent_t e, hipStream_t s);
hipError_t hipEventSynchronize(hipEvent_t e);
hipError_t hipEventElapsedTime(float* ms, hipEvent_t a, hipEvent_t b);
