"""MI355X-native Hybrid A* local planner (drop-in for planning::HybridAStar<float>)."""
