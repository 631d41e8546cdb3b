// mg_tensor.hip — the tensor-API copy kernels: SoA engine state <-> the AoS
// tensors Isaac Gym hands out (refresh_* / set_*).
//
// One thread per output element, so the AoS side (the user's tensor) is read or
// written fully coalesced; the SoA side is a per-field stride walk that the L2
// absorbs (13 fields x 4 B per row). 32-bit index math (the launchers check
// n * ncol < 2^31). An LDS-tiled transpose (64 rows per block) measured no
// faster inside the hipGraph-replayed S1 step (37.4 vs 37.5 us) and 3.5 us slower
// with 256-thread tiles: at 8192 rows these copies are launch-latency bound.
#include "mg_internal.h"

namespace {

// aos[i][f] = soa[f][ids ? ids[i] : i]
__global__ void k_gather_rows(const float* __restrict__ soa, int stride, int ncol,
                              const int* __restrict__ ids, int n, float* __restrict__ aos) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n * ncol) return;
    const int i = t / ncol;
    const int f = t - i * ncol;
    const int r = ids ? ids[i] : i;
    aos[t] = soa[(size_t)f * stride + r];
}

// the rigid-body and actor-root tensors in one launch (the paired refresh,
// migym_capi.cpp): thread (body g, field f) reads the SoA state once and writes
// rb[g][f], and root[a][f] when g is actor a's root body (body_actor[g] = a)
__global__ void k_gather_rb_root(const float* __restrict__ soa, int stride, int ncol, const int* __restrict__ perm,
                                 int nb, float* __restrict__ rb, const int* __restrict__ body_actor,
                                 float* __restrict__ root) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nb * ncol) return;
    const int g = t / ncol;
    const int f = t - g * ncol;
    const float v = soa[(size_t)f * stride + perm[g]];
    rb[t] = v;
    const int a = body_actor[g];
    if (a >= 0) root[(size_t)a * ncol + f] = v;
}

// for k < n: i = sel ? sel[k] : k;  soa[f][ids ? ids[i] : i] = aos[i][f]
// A selected row outside [0, nrows) is skipped (user indices are not trusted).
__global__ void k_scatter_rows(const float* __restrict__ aos, int ncol, const int* __restrict__ ids,
                               const int* __restrict__ sel, int n, int nrows, float* __restrict__ soa,
                               int stride) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n * ncol) return;
    const int k = t / ncol;
    const int f = t - k * ncol;
    const int i = sel ? sel[k] : k;
    if (i < 0 || i >= nrows) return;
    const int r = ids ? ids[i] : i;
    soa[(long)f * stride + r] = aos[(long)i * ncol + f];
}

// DOF rows selected by actor: for k < nsel, a = sel[k], j < count(a):
//   d = actor_dof[a] + j;  dst[c][d] = src[d][c]   (c < ncol)
// sel == null: every DOF row (nsel = num_dofs, max_dofs = 1, actor_dof unused).
// A selected actor outside [0, nactors) is skipped.
__global__ void k_scatter_dofs(const float* __restrict__ src, int ncol, const int* __restrict__ actor_dof,
                               const int* __restrict__ sel, int nsel, int nactors, int max_dofs, float* dst0,
                               float* dst1) {
    const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (long)nsel * max_dofs) return;
    int d;
    if (sel) {
        const int k = (int)(t / max_dofs);
        const int j = (int)(t - (long)k * max_dofs);
        const int a = sel[k];
        if (a < 0 || a >= nactors) return;
        const int d0 = actor_dof[a], d1 = actor_dof[a + 1];
        if (d0 + j >= d1) return;
        d = d0 + j;
    } else {
        d = (int)t;
    }
    dst0[d] = src[(long)d * ncol + 0];
    if (ncol > 1) dst1[d] = src[(long)d * ncol + 1];
}

inline int nblocks(long total, int bs) { return (int)((total + bs - 1) / bs); }

}  // namespace

hipError_t mg_launch_gather_rows(const float* soa, int stride, int ncol, const int* ids, int n,
                                 float* aos, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    if (ncol <= 0 || (long)n * ncol >= (1L << 31)) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_gather_rows, dim3(nblocks((long)n * ncol, 256)), dim3(256), 0, s,
                       soa, stride, ncol, ids, n, aos);
    return hipGetLastError();
}

hipError_t mg_launch_gather_rb_root(const float* soa, int stride, int ncol, const int* perm, int nb, float* rb,
                                    const int* body_actor, float* root, hipStream_t s) {
    if (nb <= 0) return hipSuccess;
    if (ncol <= 0 || (long)nb * ncol >= (1L << 31)) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_gather_rb_root, dim3(nblocks((long)nb * ncol, 256)), dim3(256), 0, s, soa, stride, ncol, perm,
                       nb, rb, body_actor, root);
    return hipGetLastError();
}

hipError_t mg_launch_scatter_rows(const float* aos, int ncol, const int* ids, const int* sel, int n,
                                  int nrows, float* soa, int stride, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    if (ncol <= 0 || (long)n * ncol >= (1L << 31)) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_scatter_rows, dim3(nblocks((long)n * ncol, 256)), dim3(256), 0, s,
                       aos, ncol, ids, sel, n, nrows, soa, stride);
    return hipGetLastError();
}

hipError_t mg_launch_scatter_dofs(const float* src, int ncol, const int* actor_dof, const int* sel,
                                  int nsel, int nactors, int max_dofs, float* const* dst, hipStream_t s) {
    if (nsel <= 0 || max_dofs <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_scatter_dofs, dim3(nblocks((long)nsel * max_dofs, 256)), dim3(256), 0, s,
                       src, ncol, actor_dof, sel, nsel, nactors, max_dofs, dst[0], dst[1]);
    return hipGetLastError();
}
