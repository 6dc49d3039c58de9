// The n_fft = 512 kernels of cse_enhance.hip as their own translation unit, so
// the build can give them their own code-generation flags (__graft_entry__.py).
#define CSE_ENHANCE_ONLY 512
#include "cse_enhance.hip"
