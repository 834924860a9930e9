// Host check of the units' pass ranges (bdpt_device.h bdpt_unit_range / bdpt_unit_ranges, the
// functions the kernel and the launcher share): for every launch size and unit length, with and
// without the taper, the ranges partition [0, npass) in order, each holds 1..P passes, the taper
// ends in halving ranges, and there are fewer than 256 of them (the flag tag keeps 8 bits).
#include <cstdio>
#include "../../gpu_bidirectional_raytracer_amd/csrc/bdpt_device.h"

int main() {
    const int Ps[] = {1, 2, 3, 4, 8, 16, 32, 64, 128};
    long checked = 0;
    for (int P : Ps)
        for (int npass = 1; npass <= 128; npass++)
            for (int taper = 0; taper < 2; taper++) {
                const int n = bdpt_unit_ranges(npass, P, taper);
                if (n < 1 || n > 255) { printf("FAIL count npass=%d P=%d taper=%d n=%d\n", npass, P, taper, n); return 1; }
                int pos = 0, prev = P;
                for (int r = 0; r < n; r++) {
                    int len = 0;
                    const int s = bdpt_unit_range(npass, P, taper, r, &len);
                    if (s != pos || len < 1 || len > P) {
                        printf("FAIL range npass=%d P=%d taper=%d r=%d s=%d len=%d\n", npass, P, taper, r, s, len);
                        return 1;
                    }
                    if (taper && len > prev) { printf("FAIL taper grows npass=%d P=%d r=%d\n", npass, P, r); return 1; }
                    prev = len;
                    pos += len;
                    checked++;
                }
                if (pos != npass) { printf("FAIL cover npass=%d P=%d taper=%d\n", npass, P, taper); return 1; }
            }
    printf("ok %ld ranges\n", checked);
    return 0;
}
