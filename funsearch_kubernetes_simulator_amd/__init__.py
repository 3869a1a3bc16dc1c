"""MI355X-native FunSearch Kubernetes scheduler-discovery engine."""
