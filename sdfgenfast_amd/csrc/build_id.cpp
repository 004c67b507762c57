// build_id.cpp -- the build identity of this library: SHA-256 (first 16 hex digits) of the sources
// and build files it was compiled from (sdfgenfast_amd/Makefile computes it).  bench.py reports
// PMC-derived numbers (profiles/pmc_*summary.json) only when they were measured on a library with
// the same identity (tools/pmc_summary.py stamps them).
#include "sdfgen_hip.h"

#ifndef SDFGEN_BUILD_ID
#error "SDFGEN_BUILD_ID must be defined by the Makefile"
#endif

extern "C" const char *sdfgen_hip_build_id(void) { return SDFGEN_BUILD_ID; }
