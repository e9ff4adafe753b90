# Builds the reference's ROS node source, src/local_planner.cpp, UNCHANGED against this
# repository's drop-in planner headers (TEST INFRASTRUCTURE ONLY; the boundary check of
# INTEGRATION.md §2).  Sources are compiled where they lie under $(REF); outputs go to
# oracle/_ref/ only (git-ignored, not gpurun-ignored: the prebuilt driver runs on the GPU box,
# where /root/reference does not exist).  ROS is not installed: tests/cxx/stubs/ stands in for
# ros/, tf/, std_msgs/, nav_msgs/, geometry_msgs/, perception_pkg/ and path_planning_pkg/Waypoint.h.
#   local_planner_node    local_planner.cpp as is (its own main) + lib/PedestrianHandler.cpp,
#                         linked against libhastar_amd.so: the link-level drop-in claim
#   local_planner_driver  the same with main renamed (-Dmain=...) + tests/cxx/local_planner_driver.cpp,
#                         which runs LocalPlanner<float> / LocalPlanner<double> on a scripted scenario
REF ?= /root/reference
ROOT := $(abspath $(dir $(lastword $(MAKEFILE_LIST)))/..)
OUT := $(ROOT)/oracle/_ref
LIBDIR := $(ROOT)/path_planning_pkg_amd/lib
CXX ?= g++
CXXFLAGS := -O2 -std=c++17 -ffp-contract=off
DROPIN := $(ROOT)/include/path_planning_pkg
INC := -I$(ROOT)/tests/cxx/stubs -I$(DROPIN) -I$(REF)/include/path_planning_pkg -I$(REF)/src
# the reference's PedestrianHandler (not on the planner path) over the drop-in value types
PH_INC := -include $(DROPIN)/common.h -include $(DROPIN)/Obstacle.h
LINK := -L$(LIBDIR) -lhastar_amd -Wl,-rpath,'$$ORIGIN/../../path_planning_pkg_amd/lib'
HDRS := $(wildcard $(DROPIN)/*.h) $(wildcard $(ROOT)/include/*.h) $(shell find $(ROOT)/tests/cxx/stubs -name '*.h')

all: $(OUT)/local_planner_node $(OUT)/local_planner_driver

$(OUT)/pedestrian_handler.o: $(REF)/lib/PedestrianHandler.cpp $(HDRS)
	@mkdir -p $(OUT)
	$(CXX) $(CXXFLAGS) $(INC) $(PH_INC) -c $< -o $@

$(OUT)/local_planner_node: $(REF)/src/local_planner.cpp $(OUT)/pedestrian_handler.o $(LIBDIR)/libhastar_amd.so $(HDRS)
	$(CXX) $(CXXFLAGS) $(INC) $< $(OUT)/pedestrian_handler.o $(LINK) -o $@

$(OUT)/local_planner_lib.o: $(REF)/src/local_planner.cpp $(HDRS)
	@mkdir -p $(OUT)
	$(CXX) $(CXXFLAGS) $(INC) -Dmain=reference_local_planner_main -c $< -o $@

$(OUT)/local_planner_driver: $(ROOT)/tests/cxx/local_planner_driver.cpp $(OUT)/local_planner_lib.o $(OUT)/pedestrian_handler.o $(LIBDIR)/libhastar_amd.so $(HDRS)
	$(CXX) $(CXXFLAGS) $(INC) $< $(OUT)/local_planner_lib.o $(OUT)/pedestrian_handler.o $(LINK) -o $@

clean:
	rm -rf $(OUT)
.PHONY: all clean
