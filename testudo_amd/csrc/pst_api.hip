// sqrt-PST protocol entry points (commit / open / verify) -- filled in below.
#include "../../include/tpst.h"
#include "ctx.h"

void tpst_release_pst_state(tpst_ctx*) {}
