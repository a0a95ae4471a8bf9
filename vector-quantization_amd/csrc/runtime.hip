// runtime.hip — error reporting and device queries for the libmivq C ABI.
#include "mivq_common.h"

namespace mivq {

namespace {
thread_local char g_err[1024] = "";
}

int set_error(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}

int check_launch(const char* what) {
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return set_error(MIVQ_ERR_HIP, "%s: %s", what, hipGetErrorString(e));
    return MIVQ_OK;
}

}  // namespace mivq

extern "C" const char* mivq_last_error(void) { return mivq::g_err; }

extern "C" int mivq_abi_version(void) { return MIVQ_ABI_VERSION; }

extern "C" int mivq_device_info(int device, char* name, int32_t* cus, int64_t* lds_per_cu,
                                int64_t* hbm_bytes) {
    hipDeviceProp_t p;
    const hipError_t e = hipGetDeviceProperties(&p, device);
    if (e != hipSuccess) return mivq::set_error(MIVQ_ERR_HIP, "device_info: %s", hipGetErrorString(e));
    if (name) {
        snprintf(name, 64, "%s", p.gcnArchName);
    }
    if (cus) *cus = p.multiProcessorCount;
    if (lds_per_cu) *lds_per_cu = (int64_t)p.maxSharedMemoryPerMultiProcessor;
    if (hbm_bytes) *hbm_bytes = (int64_t)p.totalGlobalMem;
    return MIVQ_OK;
}
