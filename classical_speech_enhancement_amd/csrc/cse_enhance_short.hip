// The short-hop enhance kernels of cse_enhance.hip (cse_enhance_cells_short_hop:
// n_fft 512 at hop 32 / 64, n_fft 1024 at hop 64) as their own translation
// unit, so the sweep kernels' units compile exactly as without them.
#define CSE_ENHANCE_SHORT 1
#include "cse_enhance.hip"
