// bmpc_qpplan.h -- host-side symbolic analysis of a batch of QPs sharing one sparsity
// pattern (bmpc_bandqp.h): row classification, KKT pattern, reverse Cuthill-McKee ordering,
// bandwidth and the scatter lists.  Pure C++, shared by libbmpc.so and the host build.
#pragma once

#include <string>
#include <vector>

#include "bmpc_bandqp.h"

namespace bmpc {

struct HostBandQP {
  BandQPDesc d{};   // table pointers refer to the vectors below (host copy)
  std::vector<int32_t> kind, scat, cscat, xmap, ymap;
  // everything concatenated for one device copy, in the order kind, scat, cscat, xmap, ymap
  std::vector<int32_t> blob;
  void point_tables(const int32_t* base);
};

// |v| >= this is an infinite bound (OSQP_INFTY is 1e30)
constexpr double kQPInfinity = 1e20;

// Check the bounds of every problem (no NaN, l <= u) and classify each row (equality /
// one-sided / two-sided / free), alike across the batch.  Returns "" on success.
std::string bandqp_classify(int m, int batch, const double* l, const double* u, std::vector<int>& cls);

// Validate the CSC pattern (P upper triangular, n+1 column pointers; A m x n) and the bounds
// of every problem (they must classify every row alike), then build everything.  Returns
// "" on success, else an error message.
std::string bandqp_analyse(int n, int m, const int32_t* Pp, const int32_t* Pi, const int32_t* Ap, const int32_t* Ai,
                           int batch, const double* l, const double* u, int max_iter, double eps, HostBandQP& out,
                           int cus = 256, size_t lds_per_cu = 160 * 1024);

}  // namespace bmpc
