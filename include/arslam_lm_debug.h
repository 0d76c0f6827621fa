/*
 * arslam_lm_debug.h -- component entry points of libarslam_lm.so used by the
 * parity tests to check one device stage at a time against the CPU oracle.
 * Not part of the drop-in boundary (arslam_lm.h); same error conventions.
 */
#ifndef ARSLAM_LM_DEBUG_H
#define ARSLAM_LM_DEBUG_H

#ifdef __cplusplus
extern "C" {
#endif

/* Residuals and Jacobians of n independent observations on the device.
 * cam [n*3], cap [n*6], tag [n*6], corners [n*8] -> r [n*8],
 * J [n*8*15] row-major with columns cam(3) cap(6) tag(6), as ceres'
 * AutoDiffCostFunction<ArucoReprojectionError,8,3,6,6> would produce. */
int arslam_debug_residual_jacobian(int n, const double *cam, const double *cap, const double *tag,
                                   const double *corners, double *r, double *J);

/* Dense reduced-system solve on the device: factor the lower triangle of the
 * n x n row-major SPD matrix A (in place: on return A holds L) and solve
 * A y = b.  *info = 0 on success, k+1 if pivot k was not positive. */
int arslam_debug_dense_llt(long n, double *A, const double *b, double *y, int *info);

#ifdef __cplusplus
}
#endif
#endif
