// codec_sets_d.hip -- kernel instantiations for 12..13 inputs (see codec_device.h)
#include "codec_device.h"

REDSET_DEFINE_KERNEL_SETS(kernel_sets_d, 12, make_kernel_set<12>(), make_kernel_set<13>())
