/* (float)hypot(dx, dy) of glibc == sqrtf((float)(dx^2+dy^2)) below 2^24 and
   (float)sqrt((double)(dx^2+dy^2)) above, for every 0 <= dx <= dy < 4096
   (hypot is symmetric in its arguments and their signs). The glare kernel's
   r (ipt_post.hip) relies on it. Prints the mismatch count. */
#include <math.h>
#include <stdio.h>
int main(void) {
    long bad = 0;
    for (int dy = 0; dy < 4096; ++dy)
        for (int dx = 0; dx <= dy; ++dx) {
            const float a = (float)hypot((double)dx, (double)dy);
            const long s = (long)dx * dx + (long)dy * dy;
            const float b = s < (1L << 24) ? sqrtf((float)s) : (float)sqrt((double)s);
            if (a != b) ++bad;
        }
    printf("%ld\n", bad);
    return 0;
}
