"""CPU: the walk's division by the curvature (walk_rec, csrc/pp_kernels.hip div_by) and mod2pi's
division by 2pi (csrc/pp_device.h) are bit-identical to IEEE division.  interpolate (dubins.rs:169-178) divides every point's length, sin and 1 - cos by
max_curvature c; the walk computes x / c as q = RN(x rc), then RN(q + fma(-q, c, x) rc) with
rc = RN(1 / c) — Markstein's correctly rounded quotient.  Checked here in C (gcc, FMA as the
device's v_fma_f64) for the curvatures of every scene the tests and the bench use, over the value
ranges the walk feeds it (lengths up to 2 pi n_point steps, sin, 1 - cos) and random doubles."""
import subprocess


SRC = r"""
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
static uint64_t s = 88172645463325252ull;
static uint64_t xr(void) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; }
static double u01(void) { return (double)(xr() >> 11) / 9007199254740992.0; }
int main(int argc, char** argv) {
    long long n = atoll(argv[1]), bad = 0;
    for (int a = 2; a < argc; ++a) {
        /* the walk's c = 1 / turn_radius; "2pi": mod2pi's divisor (pp_device.h) */
        const double c = argv[a][0] == '2' && argv[a][1] == 'p' ? 2.0 * 3.141592653589793
                                                               : 1.0 / atof(argv[a]);
        const double rc = 1.0 / c;
        for (long long k = 0; k < n; ++k) {
            double x;
            switch (k & 3) {
                case 0: x = (2.0 * u01() - 1.0) * 700.0; break;
                case 1: x = sin(u01() * 14.0); break;
                case 2: x = 1.0 - cos(u01() * 14.0); break;
                default: {
                    uint64_t b = xr();
                    memcpy(&x, &b, 8);
                    if (!isfinite(x) || fabs(x) > 1e300 || fabs(x) < 1e-290) continue;
                }
            }
            const double q0 = x * rc;
            const double q1 = fma(fma(-q0, c, x), rc, q0);
            if (q1 != x / c) {
                if (bad < 5) printf("c=%.17g x=%.17g: %.17g != %.17g\n", c, x, q1, x / c);
                ++bad;
            }
        }
    }
    printf("%lld\n", bad);
    return bad != 0;
}
"""


def test_division_by_curvature_is_exact(tmp_path):
    c = tmp_path / "div.c"
    c.write_text(SRC)
    exe = tmp_path / "div"
    # -ffp-contract=off: only the explicit fma() fuses, as on the device
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-o", str(exe), str(c), "-lm"], check=True)
    # turn radii of scenes.py (bench6 0.8, the fields 4.0, transit 0.8 / 3.0 in the example) and a
    # spread of others
    radii = ["0.8", "4.0", "3.0", "1.8", "1.0", "2.5", "0.3", "7.0", "0.1", "0.3333333333333333",
             "2pi"]
    r = subprocess.run([str(exe), "2000000"] + radii, capture_output=True, text=True)
    assert r.returncode == 0, r.stdout
