__version__ = "0.1.0"
__reference_version__ = "1.4.0dev"
__license__ = "Apache-2.0"
