// n_links = 6: every kernel family of this link count (fgx_ep_nl.h).
#define FGX_NL 6
#include "fgx_ep_nl.h"
