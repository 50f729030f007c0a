// n_links = 4: every kernel family of this link count (fgx_ep_nl.h).
#define FGX_NL 4
#include "fgx_ep_nl.h"
