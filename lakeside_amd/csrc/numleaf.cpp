// Numeric comparison leaves (`gt` / `ge` / `lt` / `le`): BaseExpr.filterSqlAndAccumulateFields compiles them to
// `<label> > <normalizedValue>` (BaseExpr.scala:450-459, 488-498), the value normalized per the filter's dataType:
// "duration" / "datasize" through QuantityParser.parseQuantity (core/.../utils/QuantityParser.scala:17-141, missing
// unit -> 0.0), "number" through String.toDouble, anything else NaN -- which prints as the identifier `NaN`, a DuckDB
// Binder Error, i.e. an empty glob (Commons.scala:249-253), as is a list of values for a normalized type.
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <map>
#include <regex>
#include <string>

#include "../../include/lakeside_gpu.h"
#include "evalutil.hpp"

namespace lk {

namespace {

// java.lang.Double.parseDouble on the regex-matched quantity (digits, optionally one character and digits: the
// reference's `.` is unescaped); a non-number throws NumberFormatException -> the glob's query fails.
double java_to_double(const std::string& in) {
  // Double.parseDouble's decimal grammar: surrounding whitespace, sign, NaN / Infinity, digits with an optional
  // fraction and exponent, an optional f/F/d/D suffix (hexadecimal literals are not accepted here)
  static const std::regex num("[+-]?(NaN|Infinity|([0-9]+\\.?[0-9]*|\\.[0-9]+)([eE][+-]?[0-9]+)?[fFdD]?)");
  size_t a = 0, b = in.size();
  while (a < b && static_cast<unsigned char>(in[a]) <= ' ') a++;
  while (b > a && static_cast<unsigned char>(in[b - 1]) <= ' ') b--;
  std::string q = in.substr(a, b - a);
  if (!std::regex_match(q, num)) throw PlanError(LK_ERR_ARG, "NumberFormatException: For input string: \"" + in + "\"");
  if (!q.empty() && strchr("fFdD", q.back()) && q.find("Infinity") == std::string::npos) q.pop_back();
  if (q.find("NaN") != std::string::npos) return std::numeric_limits<double>::quiet_NaN();
  if (q.find("Infinity") != std::string::npos)
    return q[0] == '-' ? -std::numeric_limits<double>::infinity() : std::numeric_limits<double>::infinity();
  return strtod(q.c_str(), nullptr);
}

// QuantityParser.parseQuantity: the first match of ([0-9]+(.[0-9]+)?)(\w+|µs); unit lower-cased; the unit's
// normalization (left-to-right Double arithmetic, as the Scala lambdas evaluate it), or none.
bool parse_quantity(const std::string& v, bool duration, double& out) {
  static const std::regex re("([0-9]+(.[0-9]+)?)(\\w+|\xC2\xB5s)");
  std::smatch m;
  if (!std::regex_search(v, m, re)) return false;
  const double x = java_to_double(m[1].str());
  std::string u = m[3].str();
  for (auto& c : u) c = char(tolower(static_cast<unsigned char>(c)));
  if (duration) {
    static const std::map<std::string, int> du = {
        {"s", 1}, {"sec", 1}, {"secs", 1}, {"second", 1}, {"seconds", 1}, {"m", 2}, {"min", 2}, {"mins", 2},
        {"minute", 2}, {"minutes", 2}, {"ms", 3}, {"milli", 3}, {"millis", 3}, {"millisecond", 3},
        {"milliseconds", 3}, {"\xC2\xB5s", 4}, {"micro", 4}, {"micros", 4}, {"microsecond", 4}, {"microseconds", 4},
        {"ns", 5}, {"h", 6}, {"hr", 6}, {"hrs", 6}, {"hour", 6}, {"hours", 6}, {"d", 7}, {"day", 7}, {"days", 7}};
    auto it = du.find(u);
    if (it == du.end()) return false;
    switch (it->second) {
      case 1: out = x * 1000000000.0; break;
      case 2: out = (x * 60) * 1000000000.0; break;
      case 3: out = x * 1000000.0; break;
      case 4: out = x * 1000.0; break;
      case 5: out = x; break;
      case 6: out = (x * 3600) * 1000000000.0; break;
      default: out = ((x * 24) * 3600) * 1000000000.0; break;
    }
    return true;
  }
  static const std::map<std::string, double> sz = {
      {"b", 1.0}, {"byte", 1.0}, {"bytes", 1.0}, {"k", 1000.0}, {"kb", 1000.0}, {"kilobyte", 1000.0},
      {"kilobytes", 1000.0}, {"m", 1e6}, {"mb", 1e6}, {"mbs", 1e6}, {"megabyte", 1e6}, {"g", 1e9}, {"gb", 1e9},
      {"gbs", 1e9}, {"gigabyte", 1e9}, {"gigabytes", 1e9}, {"t", 1e12}, {"tb", 1e12}, {"tbs", 1e12},
      {"terabyte", 1e12}, {"terabytes", 1e12}, {"pb", 1e15}, {"pbs", 1e15}, {"petabyte", 1e15}, {"petabytes", 1e15},
      {"mib", 131072.0}, {"mibs", 131072.0}, {"mebibyte", 131072.0}, {"mebibytes", 131072.0}, {"kib", 128.0},
      {"kibs", 128.0}, {"kibibyte", 128.0}, {"kibibytes", 128.0}, {"gib", 134200000.0}, {"gibs", 134200000.0},
      {"gibibyte", 134200000.0}, {"gibibytes", 134200000.0}, {"tib", 137400000000.0}, {"tibs", 137400000000.0},
      {"tibibyte", 137400000000.0}, {"tibibytes", 137400000000.0}, {"pib", 1126000000000000.0},
      {"pibs", 1126000000000000.0}, {"pibibyte", 1126000000000000.0}, {"pibibytes", 1126000000000000.0}};
  auto it = sz.find(u);
  if (it == sz.end()) return false;
  out = x * it->second;
  return true;
}

}  // namespace

bool numeric_op(const std::string& op) { return op == "gt" || op == "ge" || op == "lt" || op == "le"; }

double normalized_value(const FilterNode& f) {
  if (f.v.empty()) throw PlanError(LK_ERR_ARG, "numeric comparison without a value");
  double c = std::numeric_limits<double>::quiet_NaN();
  if (f.data_type == "number") {
    c = java_to_double(f.v[0]);
  } else if (f.data_type == "duration" || f.data_type == "datasize") {
    if (!parse_quantity(f.v[0], f.data_type == "duration", c)) c = 0.0;   // .getOrElse(0.0)
  }
  // NaN / Infinity print as identifiers (`x > NaN`): a Binder Error for every glob
  if (!std::isfinite(c)) throw PlanError(LK_ERR_ARG, "numeric comparison against " + std::to_string(c) + " (dataType " + f.data_type + ")");
  return c;
}

NumLeaf make_num_leaf(const FilterNode& f, uint32_t col, uint32_t leaf, bool& bad) {
  // the list check runs for every glob (BaseExpr.scala:450-452); the literal (normalizedValue, a lazy def) only
  // where the field exists: `bad` marks a literal whose SQL fails -- the globs holding the field come back empty
  const bool normalized = f.data_type == "duration" || f.data_type == "datasize" || f.data_type == "number";
  if (normalized && f.v.size() != 1)
    throw PlanError(LK_ERR_ARG, "filter value is a list of values for dataType: " + f.data_type);
  double c = 0.0;
  bad = false;
  try {
    c = normalized_value(f);
  } catch (const PlanError&) {
    bad = true;
  }
  NumLeaf L{};
  L.col = col;
  L.leaf = leaf;
  const double inf = std::numeric_limits<double>::infinity();
  const bool up = f.op == "gt" || f.op == "ge";   // NaN sorts greatest in DuckDB
  L.nan_pass = up ? 1u : 0u;
  L.dlo = up ? c : -inf;
  L.dhi = up ? inf : c;
  L.lo_incl = f.op == "ge" || !up;
  L.hi_incl = f.op == "le" || up;
  // integer columns: exact integer bounds when the literal prints as a decimal (|c| < 1e7, Double.toString); a
  // scientific literal is a DOUBLE in DuckDB, so the integer is cast to double first (pad = 1)
  L.pad = std::fabs(c) >= 1e7 ? 1u : 0u;
  const long long mx = std::numeric_limits<long long>::max(), mn = std::numeric_limits<long long>::min();
  auto clamp = [&](double x) -> long long {   // x integral
    if (x >= 9223372036854775808.0) return mx;
    if (x < -9223372036854775808.0) return mn;
    return (long long)x;
  };
  if (f.op == "gt") { L.ilo = c >= 9223372036854775807.0 ? mx : clamp(std::floor(c)) + 1; L.ihi = mx; if (c >= 9223372036854775807.0) L.ihi = mn; }
  else if (f.op == "ge") { L.ilo = clamp(std::ceil(c)); L.ihi = mx; if (c > 9223372036854775807.0) L.ihi = mn; }
  else if (f.op == "lt") { L.ilo = mn; L.ihi = c <= -9223372036854775808.0 ? mn : clamp(std::ceil(c)) - 1; if (c <= -9223372036854775808.0) L.ilo = mx; }
  else { L.ilo = mn; L.ihi = clamp(std::floor(c)); if (c < -9223372036854775808.0) L.ilo = mx; }
  return L;
}

}  // namespace lk
