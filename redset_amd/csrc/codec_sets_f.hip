// codec_sets_f.hip -- kernel instantiations for 15..15 inputs (see codec_device.h)
#include "codec_device.h"

REDSET_DEFINE_KERNEL_SETS(kernel_sets_f, 15, make_kernel_set<15>())
