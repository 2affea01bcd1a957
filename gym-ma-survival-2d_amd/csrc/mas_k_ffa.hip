// capacity class "ffa": <agents, heals, boxes, inventory slots, compact contact slots>
#include "mas_kernels.inc"
using CapClass_ffa = mas::Cap<4, 16, 16, 4, 8>;
MAS_INSTANTIATE(ffa, CapClass_ffa)
