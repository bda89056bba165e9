// Host-side print of every kernel family's LDS bytes per env (task_lds_bytes) and global area floats per env.
// Build: hipcc --offload-arch=gfx950 -std=c++17 -I include tools/diag/lds_sizes.hip -o /tmp/lds_sizes
#define main handarm_main_unused
#include "../../isaacgym-hand-arm_amd/csrc/handarm_hip.hip"
#undef main
#include <cstdio>
template <int FAM>
static void show(const char* name) {
    using PC = FamPhys<FAM>;
    size_t b = task_lds_bytes<PC>();
    printf("%-10s LDS %6zu B per env (%2zu workgroups per CU by LDS), global area %6d floats per env, contacts %d\n",
           name, b, (size_t)163840 / b, PC::spill_floats, PC::cap * PC::nch);
}
int main() {
    show<HA_TASK_UR5SIH>("ur5sih");
    show<FAM_UR5SIH_CLUTTER>("clutter");
    show<HA_TASK_ALLEGRO_HAND>("allegro");
    show<HA_TASK_ALLEGRO_KUKA>("kuka");
    return 0;
}
