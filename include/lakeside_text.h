/* Host-only test hook: the Java 17 Double.toString / Float.toString text the exemplar path prints for DOUBLE / FLOAT
 * columns (lakeside_amd/csrc/jdtoa.cpp; the reference gets it from DuckDB's JDBC getString, Commons.scala:428-459).
 * Built as lakeside_amd/liblakeside_text.so for the CPU differential tests; the evaluator links the same source.
 * Not part of the drop-in boundary (include/lakeside_gpu.h). */
#ifndef LAKESIDE_TEXT_H
#define LAKESIDE_TEXT_H
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Writes the NUL-terminated text of x into buf; returns its length, or -1 when cap is too small (32 always fits). */
int lk_java_double_text(double x, char* buf, size_t cap);
int lk_java_float_text(float x, char* buf, size_t cap);

#ifdef __cplusplus
}
#endif
#endif
