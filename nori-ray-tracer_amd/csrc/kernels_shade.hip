// kernels_shade.hip -- translation unit 1 of kernels.hip: k_shade and
// launch_shade (see the NORI_TU note there).
#define NORI_TU 1
#include "kernels.hip"
