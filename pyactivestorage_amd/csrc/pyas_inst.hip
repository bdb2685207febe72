// pyas_inst.hip — instantiates the kernel launchers for ONE dtype, chosen by
// -DPYAS_INST_<name>, part -DPYAS_PART=1..5 (the Makefile builds this file
// once per dtype and part).
#include "pyas_kernels.hpp"

#if defined(PYAS_INST_i8)
#define PYAS_T int8_t
#elif defined(PYAS_INST_u8)
#define PYAS_T uint8_t
#elif defined(PYAS_INST_i16)
#define PYAS_T int16_t
#elif defined(PYAS_INST_u16)
#define PYAS_T uint16_t
#elif defined(PYAS_INST_i32)
#define PYAS_T int32_t
#elif defined(PYAS_INST_u32)
#define PYAS_T uint32_t
#elif defined(PYAS_INST_i64)
#define PYAS_T int64_t
#elif defined(PYAS_INST_u64)
#define PYAS_T uint64_t
#elif defined(PYAS_INST_f32)
#define PYAS_T float
#elif defined(PYAS_INST_f64)
#define PYAS_T double
#else
#error "define PYAS_INST_<dtype>"
#endif

namespace pyas {
#if PYAS_PART == 1
PYAS_INSTANTIATE_PART1(PYAS_T)
#elif PYAS_PART == 2
PYAS_INSTANTIATE_PART2(PYAS_T)
#elif PYAS_PART == 3
PYAS_INSTANTIATE_PART3(PYAS_T)
#elif PYAS_PART == 4
PYAS_INSTANTIATE_PART4(PYAS_T)
#elif PYAS_PART == 5
PYAS_INSTANTIATE_PART5(PYAS_T)
#else
#error "define PYAS_PART=1|2|3|4|5"
#endif
}  // namespace pyas
