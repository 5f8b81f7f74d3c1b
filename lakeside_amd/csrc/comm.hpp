// Multi-GPU: one process per GPU, segments sharded across ranks, partial group tables merged over RCCL.
#pragma once
#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

#include "engine.hpp"
#include "layout.hpp"

namespace lk {

int comm_world(const Engine& E);
int comm_rank(const Engine& E);
// Element-wise max of a small host byte array across ranks (glob column unions, null flags).
void comm_allreduce_max_u8(Engine& E, uint8_t* host, size_t n);
// Concatenation, in rank order, of every rank's byte blob (variable length): one all-gather of the sizes,
// one of the blobs padded to the largest.
std::vector<std::string> comm_allgather_bytes(Engine& E, const std::string& mine);
// Reduce the partial aggregation table (P.rows/cnt/hi/lo/ext, nc cells) onto rank 0: counts by sum,
// min/max by min/max on order-preserving bits (exact), compensated sums gathered and added in rank order.
void comm_reduce_table(Engine& E, const QParams& P, int agg, size_t nc);

}  // namespace lk
