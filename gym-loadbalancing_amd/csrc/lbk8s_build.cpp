// lbk8s_build.cpp — build provenance of liblbk8s.so (include/lbk8s.h: lb_source_hash,
// lb_build_flags, lb_build_compiler).  csrc/Makefile compiles this unit with the hash of every
// source, the exact flags and the compiler version, and rebuilds it whenever a source changes.
#include "lbk8s.h"

#ifndef LBK8S_SRC_HASH
#define LBK8S_SRC_HASH "unhashed"  // built outside the Makefile
#endif
#ifndef LBK8S_BUILD_FLAGS
#define LBK8S_BUILD_FLAGS "unknown"
#endif
#ifndef LBK8S_BUILD_COMPILER
#define LBK8S_BUILD_COMPILER "unknown"
#endif

extern "C" {
const char* lb_source_hash(void) { return LBK8S_SRC_HASH; }
const char* lb_build_flags(void) { return LBK8S_BUILD_FLAGS; }
const char* lb_build_compiler(void) { return LBK8S_BUILD_COMPILER; }
}
