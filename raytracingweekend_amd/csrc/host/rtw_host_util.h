// rtw_host_util.h — error state and small helpers shared by the host library.
#pragma once
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>
#include "rtw_gpu.h"

// Record `msg` as this thread's last error and return `code`.
int rtw_fail(int code, const std::string& msg);

// malloc'd copy of a vector (nullptr for an empty one); freed with free().
template <typename T>
T* rtw_dup(const std::vector<T>& v) {
    if (v.empty()) return nullptr;
    T* p = static_cast<T*>(std::malloc(v.size() * sizeof(T)));
    std::memcpy(p, v.data(), v.size() * sizeof(T));
    return p;
}

// RTW_OK when a caller's scene desc is safe to upload, else RTW_ERR_INVALID /
// RTW_ERR_UNSUPPORTED with the reason (validate.cpp).
int validate_desc(const rtw_scene_desc* d);

// Internal entry points of the kernel translation unit (rtw_kernels.hip) for
// the host library (multi.cpp); not part of the C ABI.
int rtw_handle_device(void* handle);                                             // -1 for null
int rtw_handle_add_device(void* handle, double* dst, const double* src, size_t n);  // dst += src, synchronous
// RTW_OK when `p` is device memory of `device`, or (allow_managed) managed
// memory (hipMallocManaged), as an accum_on_device pointer; else
// RTW_ERR_INVALID naming `what`: a foreign pointer would be written by
// kernels of another GPU (a fault, or silent peer writes).  Managed memory
// is accepted where a one-GPU test covers it (rtw_render_accumulate, and
// rtw_render_multi over one GPU); rtw_render_multi over several GPUs refuses
// it (RTW_ERR_UNSUPPORTED) until a multi-GPU run covers the cross-device write.
int rtw_check_device_ptr(const void* p, int device, const char* what, bool allow_managed = true);
