// capacity class "ffal": <agents, heals, boxes, inventory slots, compact contact slots>
#include "mas_kernels.inc"
using CapClass_ffal = mas::Cap<4, 24, 16, 8, 8>;
MAS_INSTANTIATE(ffal, CapClass_ffal)
