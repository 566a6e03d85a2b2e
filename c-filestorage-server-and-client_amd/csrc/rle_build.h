// rle_build.h — which kind of build this is (the Makefile sets them; the product library sets none).
//   RLE_VARIANTS    1: the measured-slower variants kept for tests and A/B runs (the fused and
//                   resident segmented kernels, the one-pass encode, the resident small-call
//                   service, call coalescing, pipelined staging): the test library
//                   build/librle_mi355x_testhooks.so and `make variant`, never the product.
//   RLE_TEST_HOOKS  1: the drop-in's fault-injection and fake-device hooks (test library, the CPU
//                   lifecycle builds).
#pragma once
#ifndef RLE_VARIANTS
#define RLE_VARIANTS 0
#endif
#ifndef RLE_TEST_HOOKS
#define RLE_TEST_HOOKS 0
#endif
