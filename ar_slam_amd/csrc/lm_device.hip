// Device-resident LM loop: Ceres 2.0's trust-region decisions (SURVEY.md
// Appendix B; the host restatement is arslam_lm::solve in lm_solver.hip) as
// two one-thread kernels, so the host can enqueue LM iterations ahead of the
// GPU instead of waiting for each step's scalars.
//
// One iteration, all on the stream (and captured once into a hipGraph):
//   step kernels (gate_step)  -> k_lm_decide  -> copy xc -> x (accepted)
//   -> linearization kernels (gate_lin: an accepted step only) -> k_lm_finalize
//   -> copy x -> xbest (a new best point)
// k_lm_decide restates the step evaluation of TrustRegionMinimizer::Minimize
// (invalid step / ParameterToleranceReached / FunctionToleranceReached /
// IsStepSuccessful + LevenbergMarquardtStrategy::StepAccepted/StepRejected),
// k_lm_finalize FinalizeIterationAndCheckIfMinimizerCanContinue (the
// iteration record, the best point, max iterations / gradient / min radius).
// Once either sets `done`, every later kernel of the iteration and of the
// iterations already enqueued returns at once (the gates), so the host stops
// after reading the flag of a completed iteration.
#include <algorithm>
#include <cfloat>
#include <cmath>

#include "lm_internal.h"

// The decisions must round exactly as the host loop's (and Ceres' on x86):
// no fused multiply-adds (2 rho - 1, 1 - q^3 would otherwise contract).
#pragma clang fp contract(off)

namespace arslam {

namespace {

__device__ __forceinline__ unsigned long long clock100() {
  return __builtin_amdgcn_s_memrealtime();   // 100 MHz
}

__device__ __forceinline__ void set_gates(LmDevState *st) {
  st->gate_step = st->done;
  st->gate_lin = st->done || !st->need_lin;
}

__global__ void k_lm_start(LmDevState *st) {
  if (threadIdx.x == 0) {
    st->rt0 = st->rt_iter = clock100();
    set_gates(st);
  }
}

// after the step kernels: d_red holds the step's reduced scalars and flags
__global__ void k_lm_decide(LmDevState *st, const double *__restrict__ red, LmDevConsts c) {
  if (threadIdx.x != 0 || st->done) return;
  st->accept = 0;
  st->num_linear_solves++;
  arslam_lm_iteration it = st->it;
  if (red[NPART + 3] != 0.0) {   // a stuck executor wait: a device fault (the host throws)
    st->fault = 1;
    st->fault_flag = (int)red[NPART + 4];
    st->done = 1;
    set_gates(st);
    return;
  }
  const bool lin_fail = red[NPART + 2] != 0.0;   // LLT failure: Ceres' invalid step
  const bool ybad = red[P_YBAD] != 0.0 || red[NPART + 1] != 0.0;
  const double model_cost_change = red[P_MODEL];
  const bool valid = !lin_fail && !ybad && model_cost_change > 0.0;
  st->need_lin = 0;
  if (!valid) {
    // HandleInvalidStep: ++num_consecutive_invalid_steps >= max -> FAILURE (not recorded)
    if (++st->n_invalid >= c.max_invalid) {
      st->termination = ARSLAM_FAILURE;
      st->rule = ARSLAM_RULE_INVALID_STEPS;
      st->done = 1;
    } else {
      st->radius /= st->decrease_factor;   // StepIsInvalid
      st->decrease_factor *= 2.0;
      st->keep_diag = 1;
      it.cost = st->x_cost + st->fixed_cost;
      it.gradient_max_norm = st->prev_gmax;
      it.gradient_norm = st->prev_gnorm;
      it.step_is_valid = 0;
      it.step_is_successful = 0;
    }
  } else {
    st->n_invalid = 0;
    it.step_is_valid = 1;
    double candidate_cost = red[P_COST];
    if (!isfinite(candidate_cost) || red[P_CBAD] != 0.0) candidate_cost = DBL_MAX;
    it.step_norm = sqrt(red[P_STEP2] + red[NPART]);
    if (it.step_norm <= c.parameter_tolerance * (st->x_norm + c.parameter_tolerance)) {
      st->termination = ARSLAM_CONVERGENCE;
      st->rule = ARSLAM_RULE_PARAMETER;
      st->done = 1;
    } else {
      it.cost_change = st->x_cost - candidate_cost;
      if (fabs(it.cost_change) <= c.function_tolerance * st->x_cost) {
        st->termination = ARSLAM_CONVERGENCE;
        st->rule = ARSLAM_RULE_FUNCTION;
        st->done = 1;
      } else {
        it.relative_decrease = candidate_cost >= DBL_MAX ? -DBL_MAX
                                                         : (st->x_cost - candidate_cost) / model_cost_change;
        if (it.relative_decrease > c.min_relative_decrease) {
          st->accept = 1;     // x <- xc, then the linearization at it
          st->need_lin = 1;
          it.step_is_successful = 1;
          const double q = 2.0 * it.relative_decrease - 1.0;
          st->radius = fmin(c.max_radius, st->radius / fmax(1.0 / 3.0, 1.0 - q * q * q));
          st->decrease_factor = 2.0;
          st->keep_diag = 0;
        } else {
          it.step_is_successful = 0;
          st->radius /= st->decrease_factor;
          st->decrease_factor *= 2.0;
          st->keep_diag = 1;
          it.cost = candidate_cost + st->fixed_cost;
          it.gradient_max_norm = st->prev_gmax;
          it.gradient_norm = st->prev_gnorm;
        }
      }
    }
  }
  st->it = it;
  set_gates(st);
}

// after the (gated) linearization: red holds its scalars and slot norms
__global__ void k_lm_finalize(LmDevState *st, const double *__restrict__ red, LmDevConsts c) {
  if (threadIdx.x != 0 || st->done) return;
  arslam_lm_iteration it = st->it;
  st->copy_best = 0;
  if (st->need_lin) {
    const double *norms = red + 16;
    st->x_cost = red[P_COST];
    st->gmax = fmax(norms[0], norms[3]);
    st->gnorm = sqrt(norms[1] + norms[4]);
    st->x_norm = sqrt(norms[2] + norms[5]);
    it.cost = st->x_cost + st->fixed_cost;
    it.gradient_max_norm = st->gmax;
    it.gradient_norm = st->gnorm;
    st->need_lin = 0;
  }
  if (it.step_is_successful) {
    st->num_successful++;
    if (st->x_cost < st->minimum_cost) {
      st->minimum_cost = st->x_cost;
      st->copy_best = 1;
    }
  } else {
    st->num_unsuccessful++;
  }
  it.trust_region_radius = st->radius;
  const unsigned long long now = clock100();
  it.iteration_time = (double)(now - st->rt_iter) * 1e-8;
  it.cumulative_time = st->t0_s + (double)(now - st->rt0) * 1e-8;
  st->rt_iter = now;
  if (st->n_iters < kLmDevMaxIters) st->iters[st->n_iters++] = it;
  if (it.iteration >= c.max_num_iterations) {
    st->termination = ARSLAM_NO_CONVERGENCE;
    st->rule = ARSLAM_RULE_MAX_ITERS;
    st->done = 1;
  } else if (it.step_is_successful && it.gradient_max_norm <= c.gradient_tolerance) {
    st->termination = ARSLAM_CONVERGENCE;
    st->rule = ARSLAM_RULE_GRADIENT;
    st->done = 1;
  } else if (st->radius <= c.min_radius) {
    st->termination = ARSLAM_CONVERGENCE;
    st->rule = ARSLAM_RULE_MIN_RADIUS;
    st->done = 1;
  }
  st->prev_gmax = it.gradient_max_norm;
  st->prev_gnorm = it.gradient_norm;
  const int next = it.iteration + 1;
  it = arslam_lm_iteration{};
  it.iteration = next;
  st->it = it;
  set_gates(st);
}

// dst <- src when *when (the accepted candidate; a new best point)
__global__ void k_lm_copy(double *__restrict__ dst, const double *__restrict__ src, long n, const int *when) {
  if (!*when) return;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) dst[i] = src[i];
}

// test hook (arslam_lm_debug_force_indefinite) inside the device loop: the
// host loop's bit (linear solve - 1) of the mask, from the state's count
__global__ void k_lm_debug_indefinite(DevProblem P, double *S, long row, unsigned long long mask,
                                      const LmDevState *st) {
  if (threadIdx.x != 0 || gated(P.gate_step)) return;
  if (mask >> min(st->num_linear_solves, 63) & 1ull) *reduced_elem(S, P, row, row) = -1.0;
}

}  // namespace

void launch_lm_debug_indefinite(const DevProblem &P, double *S, long row, unsigned long long mask,
                                const LmDevState *st, hipStream_t s) {
  hipLaunchKernelGGL(k_lm_debug_indefinite, dim3(1), dim3(64), 0, s, P, S, row, mask, st);
}

void launch_lm_start(LmDevState *st, hipStream_t s) { hipLaunchKernelGGL(k_lm_start, dim3(1), dim3(64), 0, s, st); }

void launch_lm_decide(LmDevState *st, const double *red, const LmDevConsts &c, hipStream_t s) {
  hipLaunchKernelGGL(k_lm_decide, dim3(1), dim3(64), 0, s, st, red, c);
}

void launch_lm_finalize(LmDevState *st, const double *red, const LmDevConsts &c, hipStream_t s) {
  hipLaunchKernelGGL(k_lm_finalize, dim3(1), dim3(64), 0, s, st, red, c);
}

void launch_lm_copy(double *dst, const double *src, long n, const int *when, hipStream_t s) {
  if (n <= 0) return;
  const unsigned grid = (unsigned)std::min<long>((n + 255) / 256, 256);
  hipLaunchKernelGGL(k_lm_copy, dim3(grid), dim3(256), 0, s, dst, src, n, when);
}

}  // namespace arslam
