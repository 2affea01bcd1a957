// capacity class "2v2": <agents, heals, boxes, inventory slots, compact contact slots>
#include "mas_kernels.inc"
using CapClass_2v2 = mas::Cap<4, 4, 4, 4, 4>;
MAS_INSTANTIATE(2v2, CapClass_2v2)
