// nuts_part0.hip — NUTS kernel instantiations for layouts X(1, 1) X(16, 2) X(64, 16) (nuts_part.inc).
#define GM_NUTS_PART 0
#define GM_NUTS_PART_LAYOUTS(X) X(1, 1) X(16, 2) X(64, 16)
#include "nuts_part.inc"
