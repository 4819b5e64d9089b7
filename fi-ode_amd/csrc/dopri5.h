// Dormand-Prince 5(4) tableau of torchdiffeq 0.2.2 (RKAdaptiveStepsizeODESolver / _DORMAND_PRINCE_SHAMPINE_
// TABLEAU and DPS_C_MID), as float32 copies -- the solver casts the tableau to the state dtype --
// shared by the eval solve (odesolve.hip) and the differentiable train solve (odetrain.hip).
#pragma once

namespace fiode_dp {
namespace {                      // per translation unit (non-RDC device code)

// stage coefficients beta[i][j], i = stage 0..5 (stage 5 = c_sol: FSAL)
__device__ const float DP_BETA[6][6] = {
    {1.0f / 5, 0, 0, 0, 0, 0},
    {3.0f / 40, 9.0f / 40, 0, 0, 0, 0},
    {(float)(44.0 / 45), (float)(-56.0 / 15), (float)(32.0 / 9), 0, 0, 0},
    {(float)(19372.0 / 6561), (float)(-25360.0 / 2187), (float)(64448.0 / 6561), (float)(-212.0 / 729), 0, 0},
    {(float)(9017.0 / 3168), (float)(-355.0 / 33), (float)(46732.0 / 5247), (float)(49.0 / 176),
     (float)(-5103.0 / 18656), 0},
    {(float)(35.0 / 384), 0, (float)(500.0 / 1113), (float)(125.0 / 192), (float)(-2187.0 / 6784),
     (float)(11.0 / 84)}};

__device__ const float DP_CERR[7] = {(float)(35.0 / 384 - 1951.0 / 21600), 0, (float)(500.0 / 1113 - 22642.0 / 50085),
                                     (float)(125.0 / 192 - 451.0 / 720), (float)(-2187.0 / 6784 - -12231.0 / 42400),
                                     (float)(11.0 / 84 - 649.0 / 6300), (float)(-1.0 / 60.0)};
__device__ const float DP_CMID[7] = {(float)(6025192743.0 / 30085553152.0 / 2), 0,
                                     (float)(51252292925.0 / 65400821598.0 / 2),
                                     (float)(-2691868925.0 / 45128329728.0 / 2),
                                     (float)(187940372067.0 / 1594534317056.0 / 2),
                                     (float)(-1776094331.0 / 19743644256.0 / 2), (float)(11237099.0 / 235043384.0 / 2)};


// _select_initial_step / _optimal_step_size constants (torchdiffeq defaults for dopri5)
constexpr double DP_SAFETY = 0.9, DP_IFACTOR = 10.0, DP_DFACTOR = 0.2;

}  // namespace
}  // namespace fiode_dp
