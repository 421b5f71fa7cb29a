// ek_tpl_small_w.hip — k_small_win instantiations for rules with WHERE (see ek_tpl_small.hip).
#define EK_SW_WHERE true
#define EK_SW_FN launch_small_win_where
#include "ek_tpl_small.hip"
