/* TEST INFRASTRUCTURE: oracle libm = the system glibc float libm the reference calls. */
#include <math.h>
float orc_sinf(float x) { return sinf(x); }
float orc_cosf(float x) { return cosf(x); }
float orc_expf(float x) { return expf(x); }
float orc_logf(float x) { return logf(x); }
float orc_powf(float x, float y) { return powf(x, y); }
float orc_erff(float x) { return erff(x); }
float orc_acosf(float x) { return acosf(x); }
float orc_atan2f(float y, float x) { return atan2f(y, x); }
