// codec_sets_g.hip -- kernel instantiations for 16..16 inputs (see codec_device.h)
#include "codec_device.h"

REDSET_DEFINE_KERNEL_SETS(kernel_sets_g, 16, make_kernel_set<16>())
