// nuts_part5.hip — NUTS kernel instantiations for layouts X(32, 1) X(64, 1) X(32, 4) (nuts_part.inc).
#define GM_NUTS_PART 5
#define GM_NUTS_PART_LAYOUTS(X) X(32, 1) X(64, 1) X(32, 4)
#include "nuts_part.inc"
