// nuts_part1.hip — NUTS kernel instantiations for layouts X(2, 1) X(32, 2) X(64, 8) (nuts_part.inc).
#define GM_NUTS_PART 1
#define GM_NUTS_PART_LAYOUTS(X) X(2, 1) X(32, 2) X(64, 8)
#include "nuts_part.inc"
