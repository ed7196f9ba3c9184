"""Reusable components: component.yaml loading, lightweight Python components, component store."""
from . import _dsl_bridge
from ._component_store import ComponentStore  # noqa: F401
from ._components import (_created_task_transformation_handler, components_local_output_dir_context,  # noqa: F401
                          load_component, load_component_from_file, load_component_from_text,
                          load_component_from_url)
from ._python_op import func_to_component_file, func_to_component_text, func_to_container_op  # noqa: F401
from ._structures import ComponentSpec  # noqa: F401

_created_task_transformation_handler.append(_dsl_bridge.create_container_op_from_task)
