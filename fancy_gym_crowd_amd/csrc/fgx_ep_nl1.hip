// n_links = 1: every kernel family of this link count (fgx_ep_nl.h).
#define FGX_NL 1
#include "fgx_ep_nl.h"
