// ABI helpers shared by every entry point of libavse_hip.so.
#include "common.h"

extern "C" {

int avse_abi_version(void) { return 2; }   // 2 (round 6): out_z / dz / dx accumulate

const char* avse_strerror(int code) {
    switch (code) {
        case AVSE_OK: return "ok";
        case AVSE_EINVAL: return "invalid argument (null pointer or inconsistent optional arguments)";
        case AVSE_ESHAPE: return "unsupported shape";
        case AVSE_EDTYPE: return "unsupported dtype";
        case AVSE_ELAUNCH: return "kernel launch failed";
        case AVSE_EALIGN: return "misaligned pointer or stride";
        case AVSE_ENORESIDENT: return "grid cannot be co-resident on this device (use the single-workgroup kernels)";
        default: return "unknown error";
    }
}

}  // extern "C"
