// capacity class "1v1": <agents, heals, boxes, inventory slots, compact contact slots>
#include "mas_kernels.inc"
using CapClass_1v1 = mas::Cap<2, 4, 4, 4, 4>;
MAS_INSTANTIATE(1v1, CapClass_1v1)
