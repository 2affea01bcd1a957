// capacity class "xxl": <agents, heals, boxes, inventory slots, compact contact slots>
#include "mas_kernels.inc"
using CapClass_xxl = mas::Cap<8, 20, 16, 8, 8>;
MAS_INSTANTIATE(xxl, CapClass_xxl)
