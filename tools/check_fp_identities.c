/* Exhaustive checks of the floating-point identities the device code relies on
 * (simpleraytracing_amd/csrc/kernels/xrt_device.h), on the host's IEEE f32/f64
 * (x86-64 SSE: correctly rounded, denormals preserved):
 *   1. (float)(1.0 / (double)x) == 1.0f / x           for every f32 x   (inv_det_of, Ray.cxx:99)
 *   2. ((double)t > 1e-7) == (t > 0x1.ad7f28p-24f)    for every f32 t   (accept_t, main.cxx:687)
 *   3. round(255.0 * v / 80.0) == round(v * 3.1875)    for every f32 v in [0, 80]  (lut_u8)
 * Prints the mismatch counts; exit status 0 iff all are zero. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

static float f32(uint32_t b) { float x; memcpy(&x, &b, 4); return x; }
static uint32_t bits(float x) { uint32_t b; memcpy(&b, &x, 4); return b; }

int main(void)
{
    volatile float one = 1.0f;
    const float thr = 0x1.ad7f28p-24f;
    uint64_t bad_div = 0, bad_cmp = 0, bad_lut = 0;
    if ((double)thr > 1e-7 || (double)nextafterf(thr, 1.0f) <= 1e-7) bad_cmp++;
    for (uint64_t u = 0; u < (1ull << 32); ++u) {
        const float x = f32((uint32_t)u);
        const float a = (float)(1.0 / (double)x), c = one / x;
        if (bits(a) != bits(c) && !(isnan(a) && isnan(c))) bad_div++;
        if (((double)x > 0.0000001) != (x > thr)) bad_cmp++;
        if (x >= 0.0f && x <= 80.0f && !signbit(x)) {
            if (round(255.0 * (double)x / 80.0) != round((double)x * 3.1875)) bad_lut++;
        }
    }
    printf("inv_det mismatches %llu\naccept_t mismatches %llu\nlut mismatches %llu\n",
           (unsigned long long)bad_div, (unsigned long long)bad_cmp, (unsigned long long)bad_lut);
    return (bad_div || bad_cmp || bad_lut) ? 1 : 0;
}
