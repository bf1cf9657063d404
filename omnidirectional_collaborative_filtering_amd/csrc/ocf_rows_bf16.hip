// row-stream kernel instances for __bf16 compute (ocf_rows_impl.h)
#include "ocf_rows_impl.h"

namespace ocf {
OCF_ROWS_INSTANTIATE(__bf16)
}  // namespace ocf
