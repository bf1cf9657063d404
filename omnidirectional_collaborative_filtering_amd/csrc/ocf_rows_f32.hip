// row-stream kernel instances for float compute (ocf_rows_impl.h)
#include "ocf_rows_impl.h"

namespace ocf {
OCF_ROWS_INSTANTIATE(float)
}  // namespace ocf
