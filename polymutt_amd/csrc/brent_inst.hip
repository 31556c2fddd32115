// brent_inst.hip -- part PM_BRENT_PART of the k_brent instantiations (brent_variants.h), one object per part so the
// Makefile compiles the Brent kernel's ~130 variants in parallel; engine.hip launches them through extern declarations.
#include "engine_dev.h"
#include "brent_variants.h"

#ifndef PM_BRENT_PART
#error "compile with -DPM_BRENT_PART=<0 .. PM_BRENT_PARTS-1>"
#endif
#if PM_BRENT_PART == 0
#define PM_INST_0(...) template __global__ void k_brent<__VA_ARGS__>(DevArgs, int);
#else
#define PM_INST_0(...)
#endif
#if PM_BRENT_PART == 1
#define PM_INST_1(...) template __global__ void k_brent<__VA_ARGS__>(DevArgs, int);
#else
#define PM_INST_1(...)
#endif
#if PM_BRENT_PART == 2
#define PM_INST_2(...) template __global__ void k_brent<__VA_ARGS__>(DevArgs, int);
#else
#define PM_INST_2(...)
#endif
#if PM_BRENT_PART == 3
#define PM_INST_3(...) template __global__ void k_brent<__VA_ARGS__>(DevArgs, int);
#else
#define PM_INST_3(...)
#endif
#if PM_BRENT_PART == 4
#define PM_INST_4(...) template __global__ void k_brent<__VA_ARGS__>(DevArgs, int);
#else
#define PM_INST_4(...)
#endif
#if PM_BRENT_PART == 5
#define PM_INST_5(...) template __global__ void k_brent<__VA_ARGS__>(DevArgs, int);
#else
#define PM_INST_5(...)
#endif
#if PM_BRENT_PART == 6
#define PM_INST_6(...) template __global__ void k_brent<__VA_ARGS__>(DevArgs, int);
#else
#define PM_INST_6(...)
#endif
#if PM_BRENT_PART == 7
#define PM_INST_7(...) template __global__ void k_brent<__VA_ARGS__>(DevArgs, int);
#else
#define PM_INST_7(...)
#endif
#define PM_BRENT_X(part, ...) PM_INST_##part(__VA_ARGS__)
PM_BRENT_VARIANTS
