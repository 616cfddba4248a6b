/*
 * check.c — run-time result check printed by the drivers.
 *
 * Restates the reference's check_result (reference
 * inc/helper_functions.h:184-236): the expected y is accumulated
 * sequentially in FILE ORDER, y_ref[r] += v * x[c], and compared row by
 * row.  The reference re-parses the .mtx text for this; here the caller
 * passes the file-order entries it already read (no third parse).
 * Two criteria:
 *   abs_tol : |y - y_ref| <= abs_tol            (reference EPSILON = 1e-6,
 *                                                inc/helper_functions.h:11)
 *   rel_tol : |y - y_ref| <= rel_tol * max(|y_ref|, sum_j |a_ij| |x_j|)
 *             (SURVEY.md §8d — robust against cancellation)
 * A row fails when it violates any enabled criterion.
 */
#include <math.h>
#include <stdlib.h>

#include "spmv_host.h"

int64_t spmv_check(int64_t n_rows, int64_t nnz, const int32_t *row,
                   const int32_t *col, const double *val, const double *x,
                   const double *y, double abs_tol, double rel_tol,
                   int64_t *first_bad, double *y_ref_at_bad)
{
    double *ref = (double *)calloc((size_t)(n_rows > 0 ? n_rows : 1), sizeof(double));
    double *mag = (double *)calloc((size_t)(n_rows > 0 ? n_rows : 1), sizeof(double));
    if (!ref || !mag) {
        free(ref);
        free(mag);
        return -1;
    }
    for (int64_t i = 0; i < nnz; ++i) {
        double p = val[i] * x[col[i]];
        ref[row[i]] += p;
        mag[row[i]] += fabs(p);
    }
    int64_t bad = 0;
    if (first_bad)
        *first_bad = -1;
    for (int64_t r = 0; r < n_rows; ++r) {
        double d = fabs(y[r] - ref[r]);
        int fail = 0;
        if (abs_tol > 0.0 && !(d <= abs_tol))
            fail = 1;
        if (rel_tol > 0.0) {
            double scale = fabs(ref[r]) > mag[r] ? fabs(ref[r]) : mag[r];
            if (!(d <= rel_tol * scale))
                fail = 1;
        }
        if (fail) {
            if (bad == 0) {
                if (first_bad)
                    *first_bad = r;
                if (y_ref_at_bad)
                    *y_ref_at_bad = ref[r];
            }
            ++bad;
        }
    }
    free(ref);
    free(mag);
    return bad;
}
