// sp_libm.h -- float transcendental functions for the device path.
//
// The reference calls glibc's float libm (std::sin(float) -> sinf, ...).  Those functions are
// not correctly rounded (measured here against a double-precision evaluation: sinf/cosf differ
// on ~1.3% of inputs, logf 0.7%, erff 4.4%, acosf 7.7%), so reproducing the reference bit for
// bit needs the glibc algorithms themselves.  Each lm_* below is either an exact emulation of
// glibc 2.35's x86-64 implementation (the FMA ifunc variant where one exists), verified
// exhaustively against the host libm by tests/test_libm_exact.py, or -- where marked
// APPROX -- a double-precision evaluation rounded to float that is not yet bit-exact.
// Both the host test build and the gfx950 build compile this same code, with explicit fma()
// and no contraction, so host verification carries over to the device.
#pragma once
#include "sp_math.h"

namespace spm {

// APPROX: to be replaced by the glibc-exact emulations.
SP_HD float lm_sinf(float x) { return (float)::sin((double)x); }
SP_HD float lm_cosf(float x) { return (float)::cos((double)x); }
SP_HD float lm_expf(float x) { return (float)::exp((double)x); }
SP_HD float lm_logf(float x) { return (float)::log((double)x); }
SP_HD float lm_powf(float x, float y) { return (float)::pow((double)x, (double)y); }
SP_HD float lm_erff(float x) { return (float)::erf((double)x); }
SP_HD float lm_acosf(float x) { return (float)::acos((double)x); }

} // namespace spm
