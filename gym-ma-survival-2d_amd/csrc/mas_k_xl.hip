// capacity class "xl": <agents, heals, boxes, inventory slots, compact contact slots>
#include "mas_kernels.inc"
using CapClass_xl = mas::Cap<8, 16, 16, 8, 8>;
MAS_INSTANTIATE(xl, CapClass_xl)
