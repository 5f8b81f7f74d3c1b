// DDSketch (percentile aggregations): the host side of the `p<NN>` path.
//
// The reference builds one `DDSketches.unboundedDense(0.01)` per (time step, group-key tags) over the passing rows'
// values (PushDownAggregatorStage.scala:69-81,163-167; Aggregator.scala:28-41), ships it serialized, merges sketches
// per (timestamp, tags) in query-api (TimeGroupedSketchAggregator.scala:34-37) and reads
// getValueAtQuantile(p / 100) (BaseExpr.scala:59-61).  Library: com.datadoghq:sketches-java 0.8.2 (not vendored,
// no JVM here): its LogarithmicMapping index / value functions, DenseStore bins and quantile walk are restated below
// (published algorithm: Masson, Rim, Lee, "DDSketch", VLDB 2019).  The scan kernel bins every value on the GPU
// (dd_bin, scan_kernel.hpp); the host assembles bins into sketches (O(distinct bins)).
#pragma once
#include <cstdint>
#include <map>
#include <string>

namespace lk::dd {

constexpr double kRelativeAccuracy = 0.01;   // DDSketches.unboundedDense(0.01)

struct Mapping {             // LogarithmicMapping(0.01): index = floor(ln(v) * multiplier)
  double gamma;              // (1 + a) / (1 - a) = 1 + 2a / (1 - a)
  double multiplier;         // 1 / ln(gamma) (as 1 / log1p(gamma - 1))
  double relative_accuracy;  // (gamma - 1) / (gamma + 1)
  double min_indexable;      // Double.MIN_NORMAL * gamma: smaller magnitudes count as zero
  double max_indexable;      // Double.MAX_VALUE / gamma: larger magnitudes are untrackable (accept throws)
  // LogLikeIndexMapping.value: lowerBound(index) * (1 + relativeAccuracy), lowerBound = exp(index / multiplier)
  double value(int32_t index) const;
};
const Mapping& mapping();

struct Sketch {
  std::map<int32_t, double> pos, neg;   // index -> count (DenseStore bins, sparse here)
  double zero = 0.0;
  void add_bin(uint32_t bin, double count);   // a kernel bin id (layout.hpp DD_*)
  // DDSketch.accept(v) on the host (the kernel's dd_bin restated: |v| <= min indexable -> zero count, else
  // LogarithmicMapping.index); false for NaN / a magnitude beyond the mapping's range (checkValueTrackable throws)
  bool accept(double v);
  void merge(const Sketch& o);                // DDSketch.mergeWith: bin counts add
  double count() const;
  // DDSketch.getValueAtQuantile(q): rank = q * (count - 1); walk negative bins (descending index), the zero count,
  // positive bins (ascending); the first bin whose running count exceeds the rank gives the value.
  double quantile(double q) const;
  // DDSketch.serialize(): the DDSketch protobuf message (mapping{gamma}, positiveValues / negativeValues as dense
  // contiguousBinCounts + contiguousBinIndexOffset, zeroCount), proto3 wire format.
  std::string serialize() const;
};

}  // namespace lk::dd
