// inflate_fixed.hip -- inflate.hip built for fixed-Huffman streams (inflate_fixed_kernel).
//
// The fixed code's literal / length codes are 7-9 bits and its distance codes 5 bits, so
// 9-bit literal and 8-bit distance fast tables hold every code: 7.9 KiB of LDS per wave
// instead of 9.4 KiB, 20 waves per CU instead of 17 (the inflater is latency-bound: 12
// waves per CU cost it 20 %).  1 GiB fixed-Huffman decode: kind 1 7.55 -> 6.96 ms.  A
// dynamic-Huffman stream decodes here too (the longer codes take the canonical slow path,
// about twice as slow), so the runtime picks this kernel only on the caller's FIXED hint
// (BITAR_HIP_CODEC_DEFLATE) and inflate_kernel on DEFLATE_DYNAMIC.
#define BITAR_INFL_NS infl_fixed
#define BITAR_INFL_KERNEL inflate_fixed_kernel
#define BITAR_INFL_LIT_FAST 9
#define BITAR_INFL_DIST_FAST 8
#include "inflate.hip"
