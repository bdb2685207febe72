// pyas_inst.hip — instantiates every kernel launcher for ONE dtype, chosen
// by -DPYAS_INST_<name> (the Makefile builds this file once per dtype).
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
PYAS_INSTANTIATE_LAUNCHERS(PYAS_T)
}  // namespace pyas
