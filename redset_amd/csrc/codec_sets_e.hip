// codec_sets_e.hip -- kernel instantiations for 14..14 inputs (see codec_device.h)
#include "codec_device.h"

REDSET_DEFINE_KERNEL_SETS(kernel_sets_e, 14, make_kernel_set<14>())
