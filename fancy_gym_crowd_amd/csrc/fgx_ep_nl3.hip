// n_links = 3: every kernel family of this link count (fgx_ep_nl.h).
#define FGX_NL 3
#include "fgx_ep_nl.h"
