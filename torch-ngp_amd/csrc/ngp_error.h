#pragma once
// Error reporting shared by the host-side launchers.
int ngp_set_error(int code, const char* fmt, ...);
int ngp_check_launch(const char* what);

#define NGP_REQUIRE(cond, code, ...) \
    do {                             \
        if (!(cond)) return ngp_set_error((code), __VA_ARGS__); \
    } while (0)
