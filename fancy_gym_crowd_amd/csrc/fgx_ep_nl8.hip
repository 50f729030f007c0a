// n_links = 8: every kernel family of this link count (fgx_ep_nl.h).
#define FGX_NL 8
#include "fgx_ep_nl.h"
