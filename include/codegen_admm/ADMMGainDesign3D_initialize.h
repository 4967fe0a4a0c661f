/* ADMMGainDesign3D_initialize.h: forwards to the aclswarm_amd codegen entry points (include/aclswarm_amd_codegen.h) */
#pragma once
#include "../aclswarm_amd_codegen.h"
