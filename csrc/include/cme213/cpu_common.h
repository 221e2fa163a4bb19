// cme213x native CPU backend (g++ -O3 -fopenmp -ffp-contract=off).
// Every entry point has a C ABI and returns 0 on success.
#pragma once
#include <stdint.h>

#define CME_CPU_EXPORT extern "C" __attribute__((visibility("default")))
