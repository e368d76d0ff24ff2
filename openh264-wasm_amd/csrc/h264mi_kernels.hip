// h264mi_kernels.hip -- libh264mi: all gfx950 device code plus its host runtime and the C-ABI,
// in one translation unit (one code object; constant tables defined once).
#include "h264mi_dev.h"
#include "i4tap.inc"
#include "enc_mb.inc"
#include "enc_mb_kernel.inc"
#include "enc_bits.inc"
#include "deblock.inc"
#include "color.inc"
#include "runtime_enc.inc"
#include "capi_enc.inc"
#include "capi_dec_stub.inc"
