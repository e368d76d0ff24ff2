/* Residual-block statistics of decoded slices (tools/cavlc_stats.py; analysis only, not product code):
 * the oracle decoder (oracle/h264o_dec.c, TEST INFRASTRUCTURE) is compiled with its cavlc_read_block calls
 * routed through stat_rb, which counts per block class the blocks, TotalCoeff, trailing ones, levels and
 * the run_before codes the block needed. */
#include <stdint.h>
#include <string.h>
#include "h264o_common.h"
int cavlc_read_block(BR *r, int16_t *coef, int maxnum, int nc);
static int64_t S[3][40];  /* per class (maxnum 16 / 15 / 4): blocks, nonempty, tc, t1, levels, runs, tcHist[0..16], big levels (prefix>=3 approx |l|>3) */
void h264o_stat_reset(void) { memset(S, 0, sizeof S); }
void h264o_stat_get(int64_t *o) { memcpy(o, S, sizeof S); }
int stat_rb(BR *r, int16_t *coef, int maxnum, int nc) {
    int tc = cavlc_read_block(r, coef, maxnum, nc);
    int k = maxnum == 16 ? 0 : (maxnum == 15 ? 1 : 2);
    int64_t *s = S[k];
    s[0]++;
    if (tc > 16) tc = 16;
    s[7 + tc]++;
    if (!tc) return tc;
    s[1]++; s[2] += tc;
    int nzpos[16], n = 0, last = -1;
    for (int i = maxnum - 1; i >= 0; i--) if (coef[i]) { nzpos[n++] = i; if (last < 0) last = i; }
    int t1 = 0;
    for (int i = 0; i < n && t1 < 3; i++) { if (coef[nzpos[i]] == 1 || coef[nzpos[i]] == -1) t1++; else break; }
    s[3] += t1; s[4] += n - t1;
    for (int i = t1; i < n; i++) if (coef[nzpos[i]] > 3 || coef[nzpos[i]] < -3) s[24]++;
    int zl = last + 1 - n, runs = 0;
    for (int i = 0; i < n - 1 && zl > 0; i++) { runs++; zl -= nzpos[i] - nzpos[i + 1] - 1; }
    s[5] += runs;
    if (last + 1 - n == 0) s[6]++;  /* total_zeros 0 */
    return tc;
}
