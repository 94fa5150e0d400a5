// nuts_part4.hip — NUTS kernel instantiations for layouts X(16, 1) X(16, 4) X(64, 4) (nuts_part.inc).
#define GM_NUTS_PART 4
#define GM_NUTS_PART_LAYOUTS(X) X(16, 1) X(16, 4) X(64, 4)
#include "nuts_part.inc"
