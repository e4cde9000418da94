// k_bcem_small, the small-batch fused beta-CEM kernel (k_betacem.hip: the 20
// beta-iterations of a candidate in one workgroup), compiled in its own
// translation unit: the phase bodies are k_betacem.hip's, with the thread
// index read opaquely (tidx) so that the loop over beta-iterations does not
// keep index arithmetic of every phase live across the others.
#define MPCMMD_FUSED_TU 1
#include "k_betacem.hip"
