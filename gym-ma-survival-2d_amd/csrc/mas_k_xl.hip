// capacity class "xl": <agents, heals, boxes, inventory slots, compact contact slots>
#include "mas_kernels.inc"
using CapClass_xl = mas::Cap<8, 8, 8, 4, 8>;
MAS_INSTANTIATE(xl, CapClass_xl)
