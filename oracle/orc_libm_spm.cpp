// TEST INFRASTRUCTURE: oracle libm = the product's device libm (simplepath_amd/csrc/common/sp_libm.h)
// compiled for the host, so the GPU path can be checked bit for bit independently of how close
// that libm is to glibc (tests/test_libm_exact.py measures that separately).
#include "../simplepath_amd/csrc/common/sp_libm.h"
extern "C" {
float orc_sinf(float x) { return spm::lm_sinf(x); }
float orc_cosf(float x) { return spm::lm_cosf(x); }
float orc_expf(float x) { return spm::lm_expf(x); }
float orc_logf(float x) { return spm::lm_logf(x); }
float orc_powf(float x, float y) { return spm::lm_powf(x, y); }
float orc_erff(float x) { return spm::lm_erff(x); }
float orc_acosf(float x) { return spm::lm_acosf(x); }
float orc_atan2f(float y, float x) { return spm::lm_atan2f(y, x); }
}
