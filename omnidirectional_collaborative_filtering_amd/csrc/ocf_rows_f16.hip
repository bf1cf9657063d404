// row-stream kernel instances for _Float16 compute (ocf_rows_impl.h)
#include "ocf_rows_impl.h"

namespace ocf {
OCF_ROWS_INSTANTIATE(_Float16)
}  // namespace ocf
