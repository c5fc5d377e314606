// codec_sets_b.hip -- kernel instantiations for 7..9 inputs (see codec_device.h)
#include "codec_device.h"

REDSET_DEFINE_KERNEL_SETS(kernel_sets_b, 7, make_kernel_set<7>(), make_kernel_set<8>(), make_kernel_set<9>())
