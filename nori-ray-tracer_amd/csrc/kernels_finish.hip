// kernels_finish.hip -- translation unit 2 of kernels.hip: k_tail_prefix,
// k_finish and launch_finish (see the NORI_TU note there).
#define NORI_TU 2
#include "kernels.hip"
