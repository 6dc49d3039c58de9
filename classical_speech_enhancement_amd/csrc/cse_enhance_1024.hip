// The n_fft = 1024 kernels of cse_enhance.hip and the enhance C entry points.
#define CSE_ENHANCE_ONLY 1024
#include "cse_enhance.hip"
