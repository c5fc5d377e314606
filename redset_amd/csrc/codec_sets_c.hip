// codec_sets_c.hip -- kernel instantiations for 10..11 inputs (see codec_device.h)
#include "codec_device.h"

REDSET_DEFINE_KERNEL_SETS(kernel_sets_c, 10, make_kernel_set<10>(), make_kernel_set<11>())
