// nuts_part2.hip — NUTS kernel instantiations for layouts X(4, 1) X(64, 2) X(32, 8) (nuts_part.inc).
#define GM_NUTS_PART 2
#define GM_NUTS_PART_LAYOUTS(X) X(4, 1) X(64, 2) X(32, 8)
#include "nuts_part.inc"
