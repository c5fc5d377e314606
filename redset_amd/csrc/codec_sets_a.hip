// codec_sets_a.hip -- kernel instantiations for 1..6 inputs (see codec_device.h)
#include "codec_device.h"

REDSET_DEFINE_KERNEL_SETS(kernel_sets_a, 1, make_kernel_set<1>(), make_kernel_set<2>(), make_kernel_set<3>(), make_kernel_set<4>(), make_kernel_set<5>(), make_kernel_set<6>())
