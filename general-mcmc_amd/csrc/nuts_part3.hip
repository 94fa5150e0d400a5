// nuts_part3.hip — NUTS kernel instantiations for layouts X(8, 1) X(8, 4) X(16, 8) (nuts_part.inc).
#define GM_NUTS_PART 3
#define GM_NUTS_PART_LAYOUTS(X) X(8, 1) X(8, 4) X(16, 8)
#include "nuts_part.inc"
